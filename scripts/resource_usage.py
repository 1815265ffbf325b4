"""Per-kernel register / scratch / LDS table from hipcc's kernel-resource-usage remarks.

    python scripts/resource_usage.py [--filter darkroom] [--json out.json]

Builds the library once with -Rpass-analysis=kernel-resource-usage (gfx950, the
product flags of csrc/Makefile) into /tmp and prints one line per kernel."""
import argparse
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "decision-pretrained-transformer_amd", "csrc")
FIELDS = {"TotalSGPRs": "sgpr", "VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch",
          "Occupancy [waves/SIMD]": "occ", "LDS Size [bytes/block]": "lds",
          "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill"}


def collect(extra_flags=()):
    cmd = ["make", "-s", "-C", CSRC, "resource-usage-raw"]
    env = dict(os.environ)
    if extra_flags:
        env["EXTRA"] = " ".join(extra_flags)
    out = subprocess.run(cmd, capture_output=True, text=True, env=env)
    text = out.stdout + out.stderr
    kernels, cur = [], None
    for line in text.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            kernels.append(cur)
            continue
        if cur is None:
            continue
        for key, short in FIELDS.items():
            m = re.search(re.escape(key) + r": (\d+)", line)
            if m:
                cur[short] = int(m.group(1))
    return kernels


def demangle(names):
    try:
        out = subprocess.run(["/opt/rocm/llvm/bin/llvm-cxxfilt"], input="\n".join(names),
                             capture_output=True, text=True, check=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except Exception:
        return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filter", default="")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    ks = collect()
    for k, d in zip(ks, demangle([k["name"] for k in ks])):
        k["kernel"] = d
    ks = [k for k in ks if a.filter in k["kernel"]]
    for k in ks:
        print(f"{k.get('vgpr', 0):4d} vgpr {k.get('agpr', 0):4d} agpr {k.get('sgpr', 0):4d} sgpr "
              f"{k.get('scratch', 0):5d} B/lane scratch {k.get('occ', 0):2d} waves/SIMD "
              f"{k.get('lds', 0):6d} B lds  {k['kernel'][:150]}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(ks, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
