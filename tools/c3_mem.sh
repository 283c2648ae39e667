#!/bin/bash
# C3 on one GPU under several device budgets / fold thresholds, interleaved
# (run on the GPU box from the repo root):
#   tools/c3_mem.sh <reps> "<env settings>" ["<env settings>" ...]
# e.g. tools/c3_mem.sh 2 "" "OKM_HBM_CAP=160G" "OKM_HBM_CAP=160G OKM_FOLD_BYTES=24e9"
# One bench.py --workload c3 line per run -> gpurun_out/c3mem/<i>_<rep>.json;
# a summary (ms per job, device bytes, peak, spills) on stdout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/c3mem
mkdir -p "$OUT"
REPS=${1:?reps}
shift
for rep in $(seq 1 "$REPS"); do
    i=0
    for cfg in "$@"; do
        f="$OUT/${i}_${rep}"
        env $cfg timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample-reads 0 \
            --cpu-mt-reads 0 --no-timing > "$f.json" 2> "$f.log" || { echo "config '$cfg' failed"; tail -5 "$f.log"; exit 1; }
        python3 - "$f.json" "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d["memory"]
print(f"[{sys.argv[2] or 'default'}] {d['ms_per_step']:.1f} ms  device {m['device_bytes'] / 1e9:.1f} GB  "
      f"peak {m['device_peak_bytes'] / 1e9:.1f} GB  host {m['host_bytes'] / 1e9:.1f} GB  spills {m['spills']}  "
      f"folds {d['config']['folds_rank0']}  groups {d['config']['groups_rank0']}")
PY
        i=$((i + 1))
    done
done
