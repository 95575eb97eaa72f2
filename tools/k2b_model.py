"""CPU model of the byte-parallel K2 (csrc/qlzx_decode_bytes.hip), lane-vectorised with numpy.

A development aid: it runs the kernel's algorithm (item phase, marker ring, chunk phase with
the marker fill, pointer jumping and window/far gather) on a stream's group records as K1
emits them, so the design can be checked on CPU against the oracle's output.

usage: python tools/k2b_model.py [W] [MR]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402

TAIL = 10


def k1_groups(c: bytes):
    """GroupRecs (ip, m, a, b) and nitems as k_dec_parse emits them for a valid stream."""
    hdr = 9 if c[0] & 2 else 3
    dsize = int.from_bytes(c[5:9], "little") if hdr == 9 else c[2]
    ip, recs, n, op = hdr, [], 0, 0
    csize = len(c)
    while ip + 4 <= csize and op < dsize:
        cw = int.from_bytes(c[ip:ip + 4], "little")
        gip = ip
        ip += 4
        m = a = b = 0
        k = 0
        while k < 31 and ip < csize:
            if (cw >> k) & 1:
                t = c[ip]
                tl = 1 if t & 3 == 0 else (2 if t & 3 != 3 else (3 if t & 127 != 3 else 4))
                m |= 1 << k
                if (tl - 1) & 1:
                    a |= 1 << k
                if (tl - 1) & 2:
                    b |= 1 << k
                ip += tl
            else:
                ip += 1
            k += 1
            n += 1
        recs.append((gip, m, a, b))
        op = dsize if ip >= csize else op   # parse to the end of the stream, like K1
    return recs, n, dsize, hdr


def k1_events(c: bytes, gmax=None):
    """k_dec_parse's event loop (csrc/qlzx_decode_wave.hip), one lane: (recs, nitems, ok)."""
    hdr = 9 if c[0] & 2 else 3
    dsize = int.from_bytes(c[5:9], "little") if hdr == 9 else c[2]
    csize = len(c)
    if gmax is None:
        gmax = min(dsize, 65536) // 31 + 2
    cp = c + bytes(8)
    ip, g, gcw, mrem, extra, m, ra, rb, klast, needcw = hdr, 0, 0, 0, 0, 0, 0, 0, 31, True
    recs = []
    while True:
        kM = (mrem | 0x80000000) & -(mrem | 0x80000000)
        kM = kM.bit_length() - 1
        posM = gcw + 4 + kM + extra
        cwEnd = needcw and ip + 4 > csize
        mEnd = (not needcw) and posM >= csize
        if cwEnd:
            break
        rpos = ip if needcw else posM
        w = int.from_bytes(cp[rpos:rpos + 4], "little")
        cwEv = needcw
        mEv = (not needcw) and not mEnd
        ty = (w & 3) + (1 if (w & 127) == 3 else 0)
        code = (0x32110 >> (ty * 4)) & 15
        bad = (cwEv and ((w >> 31) == 0 or g >= gmax)) or (mEv and posM + code + 1 > csize)
        if bad:
            return recs, 0, False
        bit = 1 << kM
        ngcw = ip if cwEv else gcw
        nmrem = (w & 0x7fffffff) if cwEv else ((mrem & ~bit) if mEv else mrem)
        nextra = 0 if cwEv else (extra + code if mEv else extra)
        nm = 0 if cwEv else (m | bit if mEv else m)
        na = 0 if cwEv else (ra | bit if mEv and code & 1 else ra)
        nb = 0 if cwEv else (rb | bit if mEv and code & 2 else rb)
        ng = g + 1 if cwEv else g
        gend = ngcw + 35 + nextra
        close = (cwEv or mEv) and nmrem == 0
        partial = close and gend > csize
        if close or mEnd:
            while len(recs) < ng:
                recs.append(None)
            recs[ng - 1] = (ngcw, nm, na, nb)
        if mEnd:
            klast = kM - (posM - csize)
        elif partial:
            klast = 31 - (gend - csize)
        g, gcw, mrem, extra, m, ra, rb = ng, ngcw, nmrem, nextra, nm, na, nb
        if mEnd or partial:
            break
        if close:
            ip, needcw = gend, True
        else:
            needcw = False
    if g == 0:
        return recs, 0, False
    return recs, (g - 1) * 31 + klast, True


def decode_tok(t):
    ty = (t & 3) + ((t & 127) == 3)
    if ty == 0:
        return (t & 0xff) >> 2, 3, 1
    if ty == 1:
        return (t & 0xffff) >> 2, 3, 2
    if ty == 2:
        return (t & 0xffff) >> 6, ((t >> 2) & 15) + 3, 2
    if ty == 3:
        return (t >> 7) & 0x1ffff, ((t >> 2) & 0x1f) + 2, 3
    return t >> 15, ((t >> 7) & 255) + 3, 4


def model(c: bytes, W=4096, MR=256, k1=None):
    if k1 == "events":
        hdr = 9 if c[0] & 2 else 3
        dsize = int.from_bytes(c[5:9], "little") if hdr == 9 else c[2]
        recs, nitems, ok = k1_events(c)
        if not ok:
            return "E_CORRUPT(k1)", None
    else:
        recs, nitems, dsize, hdr = k1_groups(c)
    csize = len(c)
    cp = c + bytes(8)
    nb = (nitems + 63) // 64
    tail_from = dsize - 1 - TAIL if dsize > TAIL else 0
    win = np.zeros(W, np.uint8)
    mk = np.zeros(MR, np.int64)
    out = np.zeros(dsize + 8, np.uint8)   # the block's destination in HBM
    D, bt, tail, complete = 0, 0, False, dsize == 0
    pend = np.zeros(64, bool)
    pd = np.zeros(64, np.int64)
    pmk = np.zeros(64, np.int64)
    plit = np.zeros(64, np.int64)
    cin = 0
    c0 = 0
    while c0 < dsize:
        while True:
            if not pend.any():
                if complete or D >= c0 + 256:
                    break
                if bt >= nb:
                    return "E_CORRUPT(items ran out)", None
                lens = np.zeros(64, np.int64)
                ism = np.zeros(64, bool)
                offs = np.zeros(64, np.int64)
                tls = np.zeros(64, np.int64)
                lits = np.zeros(64, np.int64)
                pos = np.zeros(64, np.int64)
                valid = np.zeros(64, bool)
                for lane in range(64):
                    I = bt * 64 + lane
                    if I >= nitems:
                        continue
                    valid[lane] = True
                    g, k = divmod(I, 31)
                    ip, m, a, b = recs[g]
                    low = (1 << k) - 1
                    p = ip + 4 + k + bin(a & low).count("1") + 2 * bin(b & low).count("1")
                    pos[lane] = p
                    t = int.from_bytes(cp[p:p + 4], "little")
                    lits[lane] = t & 0xff
                    if (m >> k) & 1:
                        ism[lane] = True
                        offs[lane], lens[lane], tls[lane] = decode_tok(t)
                    else:
                        lens[lane], tls[lane] = 1, 1
                incl = np.cumsum(lens)
                total = int(incl[-1])
                d = D + incl - lens
                live = valid & (d < dsize)
                bad = np.zeros(64, bool)
                last = np.zeros(64, bool)
                if tail or D + total > tail_from:
                    tl_lanes = np.nonzero(live & ~ism & (d >= tail_from))[0]
                    tail_lane = 0 if tail else (int(tl_lanes[0]) if len(tl_lanes) else 64)
                    tail = tail or len(tl_lanes) > 0
                    lane_ix = np.arange(64)
                    mok = (offs >= 3) & (offs <= d) & (d + lens + 4 <= dsize) & (lane_ix < tail_lane)
                    last = live & (d + lens == dsize)
                    ip_end = pos + tls
                    eok = (ip_end == csize) | ((ip_end < hdr + 9) & (csize == hdr + 9))
                    bad = live & ((ism & ~mok) | (last & ~eok))
                else:
                    bad = ism & ((offs < 3) | (offs > d))
                if bad.any():
                    return "E_CORRUPT(check)", None
                complete = bool(last.any())
                pend = live.copy()
                pd = d.copy()
                pmk = np.where(ism, offs, 1)
                plit = lits.copy()
                D += total
                bt += 1
            wr = pend & (pd < c0 + MR)
            for lane in np.nonzero(wr)[0]:
                mk[pd[lane] & (MR - 1)] = pmk[lane]
                if pmk[lane] == 1:
                    win[pd[lane] & (W - 1)] = plit[lane]
            pend &= ~wr
            if pend.any():
                break
        # chunk phase
        p = c0 + np.arange(256)
        m = mk[(c0 & (MR - 1)) + np.arange(256)].copy()
        mk[(c0 & (MR - 1)) + np.arange(256)] = 0
        f = np.zeros(256, np.int64)
        cur = cin
        for j in range(256):
            cur = m[j] if m[j] else cur
            f[j] = cur
        cin = cur
        s = np.where(f == 1, p, p - f)
        q = (f != 1) & (s >= c0)
        sp = np.where(f == 1, 0xFFFF, s & 0xFFFF)
        while q.any():
            t = np.where(q, sp[np.clip(s - c0, 0, 255)], 0)
            lit = q & (t == 0xFFFF)
            nq = q & ~lit & (t >= c0)
            s = np.where(q & ~lit, t, s)
            q = nq
            sp = np.where(f == 1, 0xFFFF, s & 0xFFFF)
        lo = c0 + MR - W if c0 + MR > W else 0
        v = win[s & (W - 1)].copy()
        far = s < lo
        v[far] = out[s[far]]
        win[p & (W - 1)] = v
        n = min(256, dsize - c0)
        out[c0:c0 + n] = v[:n]
        c0 += 256
    return "OK", bytes(out[:dsize])


def corrupt_check(n=3000, seed=5):
    """Event-loop K1 + K2 model status/bytes == oracle on corrupted golden streams."""
    import json
    import random
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    man = json.load(open(os.path.join(root, "tests", "golden", "golden.json")))
    blob = open(os.path.join(root, "tests", "golden", "qlz_vectors.bin"), "rb").read()
    base = [blob[v["c_out"][0]:v["c_out"][0] + v["c_out"][1]] for v in man["vectors"]
            if v["cls"] in ("text", "runs", "kat") and v["n"] >= 100]
    rng = random.Random(seed)
    mism = 0
    for t in range(n):
        c = bytearray(rng.choice(base))
        if not c[0] & 1:
            continue
        hdr = 9 if c[0] & 2 else 3
        k = rng.randrange(hdr, len(c))
        c[k] = rng.randrange(256)
        c = bytes(c)
        ost, od = O.decompress(c)
        st, y = model(c, k1="events")
        ok = (st == "OK") == (ost == O.OK) and (st != "OK" or y == od)
        if not ok:
            mism += 1
            if mism < 5:
                print("mismatch", t, st, ost)
    print("corrupt cases checked:", n, "mismatches:", mism)


def solo_parse(c: bytes, gmax=None):
    """k_dec_solo's parse (csrc/qlzx_decode_solo.hip): unchecked speculative group lengths at
    every byte up to 128 B before the end, the two-group shortcut j2, the chain walk with K1's
    byte parse where there is no shortcut -> (recs, nitems, ok) like k1_events."""
    hdr = 9 if c[0] & 2 else 3
    dsize = int.from_bytes(c[5:9], "little") if hdr == 9 else c[2]
    csize = len(c)
    if gmax is None:
        gmax = min(dsize, 65536) // 31 + 2
    code = [((0x32110 >> (4 * ((b & 3) + ((b & 127) == 3)))) & 15) for b in c]
    delta = [0] * csize
    for x in range(hdr, csize):
        if x + 128 <= csize:
            cw = int.from_bytes(c[x:x + 4], "little")
            if cw >> 31:
                mrem, extra = cw & 0x7fffffff, 0
                while mrem:
                    k = (mrem & -mrem).bit_length() - 1
                    extra += code[x + 4 + k + extra]
                    mrem &= mrem - 1
                delta[x] = 35 + extra
    j2 = [0] * csize
    for x in range(hdr, csize):
        d1 = delta[x]
        d2 = delta[x + d1] if d1 and x + d1 < csize else 0
        j2[x] = d1 + d2 - 69 if d2 else 0
    x, glist, klast = hdr, [], 31
    while True:
        if x + 4 > csize:
            break
        if j2[x] and len(glist) + 2 <= gmax:
            glist += [x, x + delta[x]]
            x += j2[x] + 69
            continue
        if len(glist) >= gmax:
            return [], 0, False
        glist.append(x)
        if delta[x]:
            x += delta[x]
            continue
        cw = int.from_bytes(c[x:x + 4], "little")
        if not cw >> 31:
            return [], 0, False
        p, k = x + 4, 0
        while k < 31 and p < csize:
            cc = code[p] if (cw >> k) & 1 else 0
            if p + cc + 1 > csize:
                return [], 0, False
            p += cc + 1
            k += 1
        if k < 31:
            klast = k
            break
        x = p
    if not glist:
        return [], 0, False
    recs = []
    for g, x in enumerate(glist):
        cw = int.from_bytes(c[x:x + 4], "little")
        nk = klast if g + 1 == len(glist) else 31
        m = cw & ((1 << nk) - 1)
        mrem, extra, a, b = m, 0, 0, 0
        while mrem:
            k = (mrem & -mrem).bit_length() - 1
            pos = x + 4 + k + extra
            a |= (code[pos] & 1) << k
            b |= ((code[pos] >> 1) & 1) << k
            extra += code[pos]
            mrem &= mrem - 1
        recs.append((x, m, a, b))
    return recs, (len(glist) - 1) * 31 + klast, True


def solo_check(n=3000, seed=7):
    """solo_parse == k1_events (records, item count, status) on valid and corrupted streams."""
    import json
    import random
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    man = json.load(open(os.path.join(root, "tests", "golden", "golden.json")))
    blob = open(os.path.join(root, "tests", "golden", "qlz_vectors.bin"), "rb").read()
    base = [blob[v["c_out"][0]:v["c_out"][0] + v["c_out"][1]] for v in man["vectors"]
            if v["cls"] in ("text", "runs", "kat") and v["n"] >= 20]
    base = [b for b in base if b[0] & 1]
    rng = random.Random(seed)
    mism = 0
    for t in range(n + len(base)):
        c = bytearray(base[t] if t < len(base) else rng.choice(base))
        if t >= len(base):
            for _ in range(rng.choice((1, 1, 2, 3))):
                hdr = 9 if c[0] & 2 else 3
                k = rng.randrange(hdr, len(c))
                c[k] = rng.randrange(256)
            if rng.random() < 0.2:   # truncated (csize field rewritten to match)
                cut = rng.randrange((9 if c[0] & 2 else 3) + 1, len(c) + 1)
                c = c[:cut]
                if c[0] & 2:
                    c[1:5] = len(c).to_bytes(4, "little")
                else:
                    c[1] = len(c)
        c = bytes(c)
        r1, n1, ok1 = k1_events(c)
        r2, n2, ok2 = solo_parse(c)
        same = ok1 == ok2 and (not ok1 or (n1 == n2 and r1[:len(r2)] == r2 and len(r1) == len(r2)))
        if not same:
            mism += 1
            if mism < 5:
                print("solo mismatch", t, ok1, ok2, n1, n2, len(r1), len(r2))
    print("solo parse cases checked:", n + len(base), "mismatches:", mism)


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    MR = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    from test_gpu_decode_bytes import _cases
    bad = 0
    for k, x in enumerate(_cases()):
        c = O.compress(x)
        if not c[0] & 1:
            continue
        st, y = model(c, W, MR, k1="events")
        ok = st == "OK" and y == x
        bad += not ok
        if not ok:
            print(k, len(x), st, None if y is None else next(i for i in range(len(x)) if y[i] != x[i]))
    print("failures:", bad)


if __name__ == "__main__":
    if sys.argv[1:] == ["solo"]:
        solo_check()
        sys.exit(0)
    main()
    corrupt_check()
