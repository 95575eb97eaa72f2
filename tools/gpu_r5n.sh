#!/bin/bash
# Round 5: the c4/c5 legs over one corpus -- a small N = 1 run, then a 2-rank rehearsal on one
# GPU (gloo process group, both ranks on cuda:0); the digests of the two must match.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-r05n}; mkdir -p $O
timeout -k 10 400 python3 -u bench.py --blocks 65536 --legs-small --no-cpu --steps 3 --warmup 1 \
    > $O/n1.json 2> $O/n1.err || { echo "N=1 failed"; tail -20 $O/n1.err; exit 1; }
QLZX_BENCH_PG=gloo timeout -k 10 500 python3 -u bench.py --gpus 2 --blocks 65536 --legs-small --no-cpu --steps 3 --warmup 1 \
    > $O/n2.json 2> $O/n2.err || { echo "N=2 failed"; tail -20 $O/n2.err; exit 1; }
python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
a, b = (json.loads(open(f"{o}/{n}.json").read().strip().splitlines()[-1]) for n in ("n1", "n2"))
for leg, key in (("replay", "xor_value_crc32"), ("mixed", "xor_output_crc32")):
    print(leg, a[leg]["digest"][key], b[leg]["digest"][key], "equal" if a[leg]["digest"] == b[leg]["digest"] else "DIFFER")
PY
