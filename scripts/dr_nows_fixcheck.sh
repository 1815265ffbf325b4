#!/bin/bash
# Diagnostic (CPU side): a historic workspace-free build (scripts/dr_nows_bisect.sh worktree
# scratch/nows/<commit>) with ONLY the layer-0 query projection moved after the token-0 store (the
# round-6 fix: no MFMA result read through a branch), built next to the original as
# libdpt_hip_fix.so in scratch_run/<commit>_src (a copy that travels to the GPU box: scratch/ does
# not).  Then on the GPU: scripts/gpu_call14.sh (dr_nows_bisect.py on both libraries).
#   usage: scripts/dr_nows_fixcheck.sh <commit>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
c=$1
dst=$ROOT/scratch_run/${c}_src
rm -rf "$dst" && mkdir -p "$ROOT/scratch_run" && cp -r "$ROOT/scratch/nows/$c" "$dst"
rm -rf "$dst/.git" "$dst/tests" "$dst/profiles"
python3 - "$dst/decision-pretrained-transformer_amd/csrc/dpt_darkroom.hip" <<'PY'
import re, sys
p = sys.argv[1]
s = open(p).read()
m = re.search(r"DR_BLOCKS\(\(ln_n<NB>\(x, xn, P \+ PL::ln1_g, P \+ PL::ln1_b\),\s*u_proj3_n<NB>\(P, split0, xn, q, M\)\)\);", s)
assert m, "layer-0 site not found"
s = s[:m.start()] + "DR_BLOCKS(ln_n<NB>(x, xn, P + PL::ln1_g, P + PL::ln1_b));" + s[m.end():]
i = s.index("S.v0[d] = xn[0][k] * ydown;", m.start())
j = s.index("bar_lds();", i)
s = s[:j] + "if constexpr (!kWs) DR_BLOCKS(u_proj3_n<NB>(P, split0, xn, q, M));\n                        " + s[j:]
open(p, "w").write(s)
PY
(cd "$dst/decision-pretrained-transformer_amd/csrc" && make -s OUT=../dpt_hip/libdpt_hip_fix.so -j8)
echo "built $dst/decision-pretrained-transformer_amd/dpt_hip/libdpt_hip_fix.so"
