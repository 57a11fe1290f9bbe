#!/bin/bash
# Same-box A/B of a bench line: the working tree's library against a baseline build (ab/<lib>.so, built from
# a commit by `git worktree` + annety_amd/build.py), alternating. Usage (GPU box, repo root):
#   profiles/ab_run.sh <outdir> <baseline .so> <reps> <bench args...>
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; BASE=$2; REPS=$3; shift 3
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in $(seq 1 $REPS); do
  timeout -k 10 120 python3 bench.py "$@" > $O/new_$r.log 2>&1
  ANNETY_CRC_LIB=$GRAFT_REPO_ROOT/$BASE timeout -k 10 120 python3 bench.py "$@" > $O/base_$r.log 2>&1
done
python3 - "$O" "$REPS" <<'PY'
import json, sys
o, reps = sys.argv[1], int(sys.argv[2])
for tag in ("new", "base"):
    v = []
    for r in range(1, reps + 1):
        d = json.loads([x for x in open(f"{o}/{tag}_{r}.log") if x.startswith("{")][-1])
        v.append((d["ms_per_step"], d["roofline"]["kernel_ms_avg"], d["roofline"]["frac"]))
    print(tag, " ".join(f"{a:.4f}/{b:.4f}/{c:.4f}" for a, b, c in v))
PY
