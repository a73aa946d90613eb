"""TEST INFRASTRUCTURE ONLY: CPU restatement of the reference (see oracle/oracle.h)."""
