#!/usr/bin/env python
"""Per-kernel register / scratch / LDS / occupancy of a HIP source, from the compiler's
kernel-resource-usage remarks (no GPU needed):

  python scripts/kernel_resources.py csrc/hip/lda_gs64.hip [--filter 'gs_smallw|gs_team'] [--json OUT]
"""
import argparse
import json
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def resources(src, arch="gfx950"):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", f"--offload-arch={arch}", "-D__HIP_PLATFORM_AMD__",
           "-munsafe-fp-atomics", f"-I{os.path.join(ROOT, 'csrc', 'hip')}", "--cuda-device-only", "-c", src,
           "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.exit(r.stderr[-4000:])
    out, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?)\s*\[-Rpass-analysis", line)
        if not m:
            continue
        text = m.group(1)
        if text.startswith("Function Name:"):
            cur = {"kernel": demangle(text.split(":", 1)[1].strip())}
            out.append(cur)
        elif cur is not None and ":" in text:
            k, v = text.split(":", 1)
            cur[k.strip()] = v.strip()
    return out


def demangle(name):
    r = subprocess.run(["c++filt", name], capture_output=True, text=True)
    return (r.stdout.strip() or name).replace("oni::gs::", "").replace("(oni::GSArgs)", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default="")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = [r for r in resources(a.src) if re.search(a.filter, r["kernel"])]
    for r in rows:
        print(f"{r['kernel'][:70]:70s} vgpr {r.get('VGPRs', '?'):>4s} agpr {r.get('AGPRs', '?'):>3s} "
              f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4s} lds {r.get('LDS Size [bytes/block]', '?'):>6s} "
              f"waves/SIMD {r.get('Occupancy [waves/SIMD]', '?')}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
