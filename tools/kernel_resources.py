#!/usr/bin/env python3
"""Per-kernel register use and spills of the count kernels (wm2_count_kernel instantiations), from the
compiler's kernel-resource-usage remarks.

    python3 tools/kernel_resources.py [wm_count.hip] [-- extra hipcc flags]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def resources(src, extra=()):
    with tempfile.TemporaryDirectory() as d:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
               "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "approx_counter_amd", "csrc"),
               *extra, "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "--cuda-device-only", "-c", src,
               "-o", os.path.join(d, "k.o"), "-Rpass-analysis=kernel-resource-usage"]
        out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode:
        sys.exit(out.stderr[-2000:])
    rows, cur = [], None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|SGPRs Spill|VGPRs Spill|"
                      r"Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.split("\n")
    for r, n in zip(rows, names):
        r["name"] = n.replace("acamd::(anonymous namespace)::", "")
    return [r for r in rows if "wm2_count_kernel" in r["name"]]


def main():
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        extra = args[args.index("--") + 1:]
        args = args[:args.index("--")]
    src = args[0] if args else os.path.join(ROOT, "approx_counter_amd", "csrc", "wm_count.hip")
    print(f"{'kernel':44s} SGPR VGPR sSpill vSpill scratch occ")
    for r in resources(src, extra):
        print(f"{r['name'][:44]:44s} {r.get('TotalSGPRs', 0):4d} {r.get('VGPRs', 0):4d} {r.get('SGPRs Spill', 0):6d} "
              f"{r.get('VGPRs Spill', 0):6d} {r.get('ScratchSize [bytes/lane]', 0):7d} "
              f"{r.get('Occupancy [waves/SIMD]', 0):3d}")


if __name__ == "__main__":
    main()
