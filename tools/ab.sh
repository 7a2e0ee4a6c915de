#!/bin/bash
# A/B the bench across variants on one box, interleaved to spread drift:
#   bash tools/ab.sh TAG ROUNDS VARIANT [VARIANT ...] [-- extra bench.py args]
# A VARIANT is "-" (the tree as is) or space-separated environment settings
# and bench.py flags, e.g. "GSR_FIRST_MAJOR_ALONE=1", "GSR_LIB_PATH=varlib/x.so
# GSR_CHUNK=128" or "--inflight 20 --share 10".
# Each run: python bench.py --no-cpu-baseline (+ extra args) under its own time
# limit; results in gpurun_out/TAG/<variant index>_<round>.json and one summary
# line per run on stdout.  The first failing run ends the script.
TAG=$1
ROUNDS=$2
shift 2
VARIANTS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
    VARIANTS+=("$1")
    shift
done
[ "$1" = "--" ] && shift
EXTRA="$*"
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 "$ROUNDS"); do
    for i in "${!VARIANTS[@]}"; do
        v=${VARIANTS[$i]}
        envs=()
        args=()
        if [ "$v" != "-" ]; then
            read -r -a toks <<< "$v"
            for t in "${toks[@]}"; do
                if [[ "$t" == --* ]] || [ ${#args[@]} -gt 0 ]; then args+=("$t"); else envs+=("$t"); fi
            done
        fi
        out=$O/${i}_$r.json
        timeout -k 10 240 env "${envs[@]}" python bench.py --no-cpu-baseline $EXTRA "${args[@]}" > $out 2> $O/${i}_$r.err
        rc=$?
        if [ $rc -ne 0 ]; then
            echo "[ab] variant $i ($v) round $r FAILED rc=$rc"
            exit $rc
        fi
        python - "$out" "$i" "$v" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
st = {k: round(v * 1e3, 1) for k, v in (d.get("stage_ms") or {}).items()}
print(f"[ab] {sys.argv[2]} ({sys.argv[3]}): ms/frame {d['ms_per_step']:.4f} latency {d['latency_ms_per_frame']:.4f} "
      f"median {d['latency_ms_median']:.4f} stages {st}", flush=True)
EOF
    done
done
