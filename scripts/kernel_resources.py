"""Per-kernel resource usage of a HIP source built for gfx950 (CPU only):
VGPRs, AGPRs, SGPRs, scratch bytes, LDS bytes and occupancy from the
compiler's -Rpass-analysis=kernel-resource-usage remarks.  A frame instance
that suddenly needs scratch (private memory) runs several times slower; this
catches it before a GPU run.

    python scripts/kernel_resources.py stochquant_amd/csrc/sq_phi4.hip [--filter tb2]
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize", "VGPRs Spill", "Occupancy", "LDS Size")


def resources(src, extra=()):
    sys.path.insert(0, ROOT)
    from stochquant_amd.build import COMMON, HIPCC, ARCH
    cmd = [HIPCC] + COMMON + [f"--offload-arch={ARCH}", "-x", "hip", "-c", src, "-o", os.devnull,
                              "-Rpass-analysis=kernel-resource-usage"] + list(extra)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-4000:])
    return parse(r.stderr)


def parse(text):
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+) \[", line)
        if m and cur and m.group(1) in KEYS:
            out[cur][m.group(1)] = int(m.group(2))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default="")
    ap.add_argument("--remarks", help="parse this saved remark text instead of compiling")
    a = ap.parse_args()
    res = parse(open(a.remarks).read()) if a.remarks else resources(a.src)
    for name, d in sorted(res.items()):
        if a.filter in name:
            print(" ".join(f"{k}={d.get(k)}" for k in KEYS), name[:100])


if __name__ == "__main__":
    main()
