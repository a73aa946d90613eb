"""Summarise `hipcc -Rpass-analysis=kernel-resource-usage` output, one line per kernel."""
import re
import sys

KEYS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("TotalSGPRs", "sgpr"),
        (r"ScratchSize \[bytes/lane\]", "scratch"), (r"Occupancy \[waves/SIMD\]", "occ"),
        ("VGPRs Spill", "vspill"), ("SGPRs Spill", "sspill")]


def main(path):
    txt = open(path).read()
    for b in txt.split("Function Name: ")[1:]:
        name = b.split()[0]
        m = re.search(r"(\w+?)_kernelI([fd])Li(\d+)ELb(\d)", name)
        label = f"{m.group(1):8s} {m.group(2)} N={int(m.group(3)):2d} fast={m.group(4)}" if m else name[:40]
        vals = []
        for k, short in KEYS:
            mm = re.search(k + r": (\d+)", b)
            vals.append(f"{short}={mm.group(1) if mm else '?':>4}")
        print(label, " ".join(vals))


if __name__ == "__main__":
    main(sys.argv[1])
