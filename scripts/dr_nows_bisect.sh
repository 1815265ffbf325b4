#!/bin/bash
# Diagnostic (CPU side): build the library of historic commits with the workspace-free DarkRoom
# kernel's step specialised on the block count, the change that was once recorded as giving wrong
# logits (round 5, DESIGN.md "workspace-free kernels").  Each commit goes to a detached worktree
# under scratch/nows/<commit>; in commits before d33572b the workspace-free kernel took the
# run-time dispatch, and the patch turns the `if constexpr (kWs)` around the specialised calls into
# `if constexpr (true)`.  Run the comparison on the GPU with scripts/dr_nows_bisect.py.
#   usage: scripts/dr_nows_bisect.sh <commit>...   (-j: builds run 4 at a time)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
mkdir -p scratch/nows
build_one() {
    c=$1
    wt=scratch/nows/$c
    if [ ! -d "$wt" ]; then git worktree add --detach "$wt" "$c" > /dev/null 2>&1; fi
    src=$wt/decision-pretrained-transformer_amd/csrc/dpt_darkroom.hip
    # the dispatch of the step's forward (as d33572b did; the episode prologue keeps its dispatch)
    python3 - "$src" <<'EOF'
import re, sys
p = sys.argv[1]
s = open(p).read()
n = 0
for pat in (r"if constexpr \(kWs\) \{\n(\s*)if \(nb == 2\) forward",):
    s, k = re.subn(pat, lambda m: m.group(0).replace("if constexpr (kWs)", "if constexpr (true)"), s)
    n += k
s = s.replace("#define DPT_DR_SPEC_NOWS 0", "#define DPT_DR_SPEC_NOWS 1")
open(p, "w").write(s)
print(p, "patched dispatch sites:", n)
EOF
    (cd "$wt/decision-pretrained-transformer_amd/csrc" && make -s > "$ROOT/scratch/nows/$c.build.log" 2>&1) &&
        echo "$c built" || echo "$c BUILD FAILED"
}
i=0
for c in "$@"; do
    build_one "$c" &
    i=$((i + 1))
    if [ $((i % 4)) -eq 0 ]; then wait; fi
done
wait
