#!/bin/bash
# Round 4: kernel trace of 16 concurrent qlz_decompress callers (16 KiB), to see the coalescing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04t}; mkdir -p $O
gcc -O2 -pthread -o $O/mt_single tools/mt_single.c -ldl || exit 1
python3 - $O <<'PY' || exit 1
import sys; sys.path.insert(0, '.')
from oracle import oracle as O
open(sys.argv[1] + '/c16384.bin', 'wb').write(O.compress(O.gen_text(0x5EED2026, 16384, 16384)))
PY
timeout -k 10 60 $O/mt_single $PWD/gobeansdb_amd/libqlzx.so $O/c16384.bin 16 1 | tee $O/mt.jsonl || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o trace -- $O/mt_single $PWD/gobeansdb_amd/libqlzx.so $O/c16384.bin 16 1 > $O/mt_traced.jsonl 2>&1 || { tail $O/mt_traced.jsonl; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, statistics
f = glob.glob(sys.argv[1] + '/trace/**/*kernel_trace.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if 'svc_decode' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows]
g = [(int(b['Start_Timestamp']) - int(a['Start_Timestamp'])) / 1e3 for a, b in zip(rows, rows[1:])]
wg = [int(r.get('Grid_Size', r.get('Grid_Size_X', 0)) or 0) for r in rows]
print('kernels', len(rows), 'median dur us', statistics.median(d), 'p90', sorted(d)[int(0.9 * len(d))],
      'median start gap us', statistics.median(g), 'grid sizes (median)', statistics.median(wg) if wg else None)
print('keys', list(rows[0].keys()))
PY
