"""Per-call latency of the single-call drop-ins (qlz_compress, qlz_decompress, crc32_write)
against the reference C build (oracle/_ref) called the same way, one call at a time.

These are the calls store/ makes per value: CCompress once or twice per set
(store/item.go:140,151), crc32.write three times per record (store/datafile.go:68-74),
CDecompressSafe per get (store/item.go:167).  Every call goes through ctypes on both sides,
so the Python call overhead (~1 us) is in both columns.  The reference column "cgo" also
allocates a 528,400-B scratch and the output buffer per call, as cquicklz.go:24-34 does.
Each size has --values DISTINCT text values (1024 by default) and consecutive calls take the
next one, on both sides: no call repeats the previous call's value, so neither side gets a
warmed branch predictor or cache from decoding one value in a loop.

usage: python tools/bench_single.py [--calls 1000] [--values 1024] [--out FILE] [--dump DIR]
  --dump DIR writes DIR/values_<n>.bin for tools/mt_single.c
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def med_us(fn, calls, pct=None):
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter_ns()
        fn()
        ts.append(time.perf_counter_ns() - t0)
    if pct is not None:
        pct["p99"] = round(float(np.percentile(ts, 99)) / 1e3, 2)
    return round(float(np.median(ts)) / 1e3, 2)


def aggregate(fn_for_thread, threads, seconds):
    """Calls/s of `threads` threads each calling its own fn in a loop (ctypes drops the GIL)."""
    import threading
    stop = threading.Event()
    counts = [0] * threads
    fns = [fn_for_thread(t) for t in range(threads)]

    def worker(t):
        f = fns[t]
        c = 0
        while not stop.is_set():
            f()
            c += 1
        counts[t] = c

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    time.sleep(seconds)
    stop.set()
    for th in ths:
        th.join()
    return sum(counts) / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=1000)
    ap.add_argument("--values", type=int, default=1024, help="distinct values per size")
    ap.add_argument("--out", default=None)
    ap.add_argument("--dump", default=None, help="write values_<n>.bin (tools/mt_single.c input) here")
    ap.add_argument("--threads", type=int, default=16, help="aggregate-throughput callers (0: skip)")
    ap.add_argument("--seconds", type=float, default=3.0)
    a = ap.parse_args()
    from gobeansdb_amd import _lib
    from oracle import oracle as O
    L = _lib.lib()
    ref = O.ref()
    rows = []
    # a 20-B crc32_write (the header slice of every record read and write)
    h20 = [np.frombuffer(os.urandom(20), np.uint8).copy() for _ in range(a.values)]
    for hh in h20:
        assert L.crc32_write(0xFFFFFFFF, hh.ctypes.data, 20) == O.crc32_write(0xFFFFFFFF, hh.tobytes())
    st_ = [0]

    def c20(lib):
        def f():
            k = st_[0]
            st_[0] = k + 1 if k + 1 < a.values else 0
            lib.crc32_write(0xFFFFFFFF, h20[k].ctypes.data, 20)
        return f
    row20 = {"bytes": 20, "gpu_lib_crc32_us": med_us(c20(L), a.calls)}
    if ref is not None:
        row20["ref_crc32_us"] = med_us(c20(ref[1]), a.calls)
    rows.append(row20)
    print(json.dumps(row20), flush=True)
    for n in (4096, 16384, 65536):
        plains = [O.gen_text(0x5EED2026 + n, i, n) for i in range(a.values)]
        comps = [O.compress(p) for p in plains]
        if a.dump:
            import struct
            with open(os.path.join(a.dump, f"values_{n}.bin"), "wb") as f:
                for c, p in zip(comps, plains):
                    f.write(struct.pack("<II", len(c), len(p)) + c + p)
        src = [np.frombuffer(p, np.uint8).copy() for p in plains]
        csrc = [np.frombuffer(c, np.uint8).copy() for c in comps]
        dst = np.zeros(n + 400, np.uint8)
        scratch = np.zeros(528400, np.uint8)
        # correctness of the GPU side on every value before timing
        for k in range(a.values):
            assert L.qlz_compress(src[k].ctypes.data, dst.ctypes.data, n, scratch.ctypes.data) == len(comps[k])
            assert dst[:len(comps[k])].tobytes() == comps[k]
            assert L.qlz_decompress(csrc[k].ctypes.data, dst.ctypes.data, scratch.ctypes.data) == n
            assert dst[:n].tobytes() == plains[k]
            assert L.crc32_write(0xFFFFFFFF, src[k].ctypes.data, n) == O.crc32_write(0xFFFFFFFF, plains[k])
        row = {"bytes": n, "values": a.values, "ratio": round(sum(map(len, comps)) / (n * a.values), 3)}
        nv = a.values

        def cyc(f):
            """f(k) over the values in turn"""
            state = [0]

            def g():
                k = state[0]
                state[0] = k + 1 if k + 1 < nv else 0
                f(k)
            return g

        row["gpu_compress_us"] = med_us(cyc(lambda k: L.qlz_compress(src[k].ctypes.data, dst.ctypes.data, n, 0)),
                                        a.calls)
        pct = {}
        row["gpu_decompress_us"] = med_us(cyc(lambda k: L.qlz_decompress(csrc[k].ctypes.data, dst.ctypes.data, 0)),
                                          a.calls, pct)
        row["gpu_decompress_p99_us"] = pct["p99"]
        row["gpu_crc32_us"] = med_us(cyc(lambda k: L.crc32_write(0xFFFFFFFF, src[k].ctypes.data, n)), a.calls)
        if ref is not None:
            Q, C = ref

            def cgo_compress(k):
                sc = np.empty(528400, np.uint8)
                out = np.empty(n + 400, np.uint8)
                Q.qlz_compress(src[k].ctypes.data, out.ctypes.data, n, sc.ctypes.data)

            def cgo_decompress(k):
                out = np.empty(n, np.uint8)
                Q.qlz_decompress(csrc[k].ctypes.data, out.ctypes.data, scratch.ctypes.data)

            row["ref_compress_us"] = med_us(cyc(lambda k: Q.qlz_compress(src[k].ctypes.data, dst.ctypes.data, n,
                                                                         scratch.ctypes.data)), a.calls)
            row["ref_compress_cgo_us"] = med_us(cyc(cgo_compress), a.calls)
            row["ref_decompress_us"] = med_us(cyc(lambda k: Q.qlz_decompress(csrc[k].ctypes.data, dst.ctypes.data,
                                                                             scratch.ctypes.data)), a.calls)
            row["ref_decompress_cgo_us"] = med_us(cyc(cgo_decompress), a.calls)
            row["ref_crc32_us"] = med_us(cyc(lambda k: C.crc32_write(0xFFFFFFFF, src[k].ctypes.data, n)), a.calls)
        # one GET as readRecordAt + Payload.Decompress make it (store/datafile.go:161-168,
        # store/item.go:163-176) on a record with a compressed value: three crc32_write slices
        # (header[4:24], key, value) then the decode; with qlzx_read_record1 the value's CRC and the
        # decode are one request.  Correctness first, on every record.
        from oracle import replay as R
        recs = []
        for k in range(nv):
            key = b"key_%016x" % k
            rec = R.make_record(key, comps[k], flag=R.FLAG_COMPRESS, ver=1)
            recs.append((np.frombuffer(rec[4:24], np.uint8).copy(), np.frombuffer(key, np.uint8).copy(),
                         int.from_bytes(rec[:4], "little")))
        out_len = ctypes.c_size_t(0)
        st32 = ctypes.c_int32(0)

        def get_drop_ins(k, lib=L):
            h, key, crc = recs[k]
            s_ = lib.crc32_write(0xFFFFFFFF, h.ctypes.data, 20)
            s_ = lib.crc32_write(s_, key.ctypes.data, len(key))
            s_ = lib.crc32_write(s_, csrc[k].ctypes.data, len(comps[k]))
            assert s_ ^ 0xFFFFFFFF == crc
            return lib.qlz_decompress(csrc[k].ctypes.data, dst.ctypes.data, scratch.ctypes.data)

        def get_one_request(k):
            h, key, crc = recs[k]
            s_ = L.crc32_write(0xFFFFFFFF, h.ctypes.data, 20)
            s_ = L.crc32_write(s_, key.ctypes.data, len(key))
            L.qlzx_read_record1(csrc[k].ctypes.data, len(comps[k]), s_, crc, 1, dst.ctypes.data, n,
                                ctypes.byref(out_len), ctypes.byref(st32))
        for k in range(nv):
            assert get_drop_ins(k) == n and dst[:n].tobytes() == plains[k]
            dst[:] = 0
            get_one_request(k)
            assert st32.value == 0 and out_len.value == n and dst[:n].tobytes() == plains[k]
        row["gpu_get_drop_ins_us"] = med_us(cyc(get_drop_ins), a.calls)
        row["gpu_get_read_record1_us"] = med_us(cyc(get_one_request), a.calls)
        if ref is not None:
            Cq = ref[1]

            class _Ref:  # the reference crc32_write and qlz_decompress, called the same way
                crc32_write = Cq.crc32_write
                qlz_decompress = ref[0].qlz_decompress
            row["ref_get_us"] = med_us(cyc(lambda k: get_drop_ins(k, _Ref)), a.calls)
        if a.threads:
            def mk(lib):
                def for_thread(t):
                    out = np.zeros(n + 64, np.uint8)
                    sc = np.zeros(528400, np.uint8)
                    state = [t * nv // a.threads]

                    def call():
                        k = state[0]
                        state[0] = k + 1 if k + 1 < nv else 0
                        lib.qlz_decompress(csrc[k].ctypes.data, out.ctypes.data, sc.ctypes.data)
                    return call
                return for_thread
            cps = aggregate(mk(L), a.threads, a.seconds)
            row["gpu_decompress_threads"] = a.threads
            row["gpu_decompress_agg_GiBps"] = round(cps * n / 2**30, 3)
            row["gpu_decompress_agg_calls_per_s"] = round(cps)
            if ref is not None:
                cps = aggregate(mk(ref[0]), a.threads, a.seconds)
                row["ref_decompress_agg_GiBps"] = round(cps * n / 2**30, 3)
        rows.append(row)
        print(json.dumps(row), flush=True)
    res = {"what": "median per-call latency, one call at a time (ctypes on both sides), text values, each call "
                   "on the next of --values distinct values; agg_*: aggregate qlz_decompress rate of --threads "
                   "concurrent Python callers (tools/mt_single.c gives the pthread figure)",
           "calls_per_point": a.calls, "values_per_size": a.values, "rows": rows,
           "reference": "oracle/_ref (quicklz.c, crc32.go preamble; gcc -O2)" if ref else None}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
