#!/bin/bash
# GPU-box recipe for committed profiles of one bench workload: a kernel trace
# (--kernel-trace --stats) of the bench command itself (its own printed bench line is checked
# against its trace by tools/trace_check.py) and four separate PMC passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass; SQ and GRBM counters in their own).  Each step is
# time-limited; the chain stops at the first fault / timeout (tools/gpu_steps.sh).  A fifth pass
# counts the VALU FLOPs the kernel executes (SQ_INSTS_VALU_FLOPS_FP32/FP64, gfx950) for roofline.valu.
#
# usage (via gpurun): tools/profile_round.sh TAG [bench.py args...]
#   outputs under gpurun_out/TAG/{trace,pmc_fetch,pmc_write,pmc_sq,pmc_grbm} + TAG_*.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$PWD
TAG=${1:?usage: profile_round.sh TAG [bench args]}
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
B="python3 $R/bench.py --no-cpu-baseline --no-secondary --steps ${PROF_STEPS:-300} $*"
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "${TAG}_trace" 300 "cd /tmp && rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B" \
  "${TAG}_pmc_fetch" 300 "cd /tmp && rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B" \
  "${TAG}_pmc_write" 300 "cd /tmp && rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B" \
  "${TAG}_pmc_sq" 300 "cd /tmp && rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_sq -o run --output-format csv -- $B" \
  "${TAG}_pmc_grbm" 300 "cd /tmp && rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS -d $O/pmc_grbm -o run --output-format csv -- $B" \
  "${TAG}_pmc_flops" 300 "cd /tmp && rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES -d $O/pmc_flops -o run --output-format csv -- $B"
