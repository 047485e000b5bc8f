#!/usr/bin/env python3
"""One line per bench log of an A/B directory: ms_per_step and the step-time spread.

    python tools/ab_table.py gpurun_out/r04_m2
"""
import glob
import json
import os
import sys


def main():
    for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
        for line in open(f, errors="replace"):
            if line.startswith("{"):
                try:
                    d = json.loads(line)
                except ValueError:
                    continue
                if "ms_per_step" not in d:
                    continue
                st = d.get("step_ms", {})
                print(f"{os.path.basename(f)[:-4]:28s} ms {d['ms_per_step']:.4f}  p50 {st.get('p50', 0):.4f}  "
                      f"min {st.get('min', 0):.4f}  max {st.get('max', 0):.3f}")


if __name__ == "__main__":
    main()
