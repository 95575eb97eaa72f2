"""Assemble the single-call profile from a GPU run (latency table, phase stamps, 1/16-thread
aggregate) and the reference's aggregate (mt.jsonl lines of oracle/_ref's library), which round 5's
tools/gpu_r5s.sh writes into the same directory (round 4: tools/gpu_r4j.sh + gpu_r4c.sh).
usage: python tools/collect_single.py RUN_DIR REF_RUN_DIR OUT.json [round=5]
"""
import json
import sys

run, refrun, out = sys.argv[1:4]
rnd = int(sys.argv[4]) if len(sys.argv) > 4 else 5
lat = json.load(open(f"{run}/single_call.json"))
mt = [json.loads(x) for x in open(f"{run}/mt.jsonl") if "qlzref" not in x]
mt_ref = [json.loads(x) for x in open(f"{refrun}/mt.jsonl") if "qlzref" in x]
agg = []
for r in mt:
    ref = [q for q in mt_ref if q["threads"] == r["threads"] and q["dsize"] == r["dsize"]]
    agg.append({"dsize": r["dsize"], "threads": r["threads"], "gpu_GiBps": r["GiBps"],
                "gpu_us_per_call_per_thread": r["us_per_call_per_thread"],
                "ref_GiBps": ref[0]["GiBps"] if ref else None,
                "ref_us_per_call_per_thread": ref[0]["us_per_call_per_thread"] if ref else None})
row16 = [r for r in lat["rows"] if r["bytes"] == 16384][0]
a16 = [a for a in agg if a["dsize"] == 16384 and a["threads"] == 16][0]
p50_bar, agg_bar = (35, 8.0) if rnd >= 5 else (30, None)
res = {
    "what": "single-call drop-ins (qlz_decompress / qlz_compress / crc32_write) on one MI355X: per-call "
            "latency (one caller), aggregate qlz_decompress of 1 and 16 pthreads (tools/mt_single.c), and the "
            "small-block decoder's phase stamps (core cycles, qlzx_decode_small.hip); every call on the next of "
            "1024 distinct values per size, on both sides",
    "command": "tools/gpu_r5s.sh" if rnd >= 5 else "tools/gpu_r4j.sh + tools/gpu_r4c.sh",
    "latency": lat,
    "aggregate_qlz_decompress": agg,
    "phase_stamps": open(f"{run}/solo_prof.txt").read().splitlines(),
    "targets": {
        "p50_qlz_decompress_16KiB_us": {"target": p50_bar, "measured": row16["gpu_decompress_us"],
                                        "met": row16["gpu_decompress_us"] <= p50_bar},
        "aggregate_16_threads_16KiB_GiBps": {"target": agg_bar if agg_bar else "reference 16-thread rate",
                                             "measured": a16["gpu_GiBps"], "reference_same_box": a16["ref_GiBps"],
                                             "met": a16["gpu_GiBps"] >= (agg_bar or (a16["ref_GiBps"] or 1e9))},
    },
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["targets"]))
