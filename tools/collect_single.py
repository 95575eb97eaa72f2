"""Assemble profiles/r04_single_call.json from a tools/gpu_r4j.sh run (latency table, phase stamps,
16-thread aggregate) and the reference's aggregate from tools/gpu_r4c.sh on the same box type.
usage: python tools/collect_single.py gpurun_out/r04j5 gpurun_out/r04c profiles/r04_single_call.json
"""
import json
import sys

run, refrun, out = sys.argv[1:4]
lat = json.load(open(f"{run}/single_call.json"))
mt = [json.loads(x) for x in open(f"{run}/mt.jsonl")]
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
res = {
    "what": "single-call drop-ins (qlz_decompress / qlz_compress / crc32_write) on one MI355X: per-call "
            "latency (one caller), aggregate qlz_decompress of 1 and 16 pthreads (tools/mt_single.c), and the "
            "small-block decoder's phase stamps (core cycles, qlzx_decode_small.hip)",
    "latency": lat,
    "aggregate_qlz_decompress": agg,
    "phase_stamps": open(f"{run}/solo_prof.txt").read().splitlines(),
    "targets": {
        "p50_qlz_decompress_16KiB_us": {"target": 30, "measured": row16["gpu_decompress_us"],
                                        "met": row16["gpu_decompress_us"] <= 30},
        "aggregate_16_threads_GiBps": {"target": "reference 16-thread rate", "measured": a16["gpu_GiBps"],
                                       "reference_same_box": a16["ref_GiBps"],
                                       "met": a16["ref_GiBps"] is not None and a16["gpu_GiBps"] >= a16["ref_GiBps"]},
    },
    "round3_16KiB_decompress_us": 97,
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["targets"]))
