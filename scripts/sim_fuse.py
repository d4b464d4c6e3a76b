"""CPU walk-through of k_fuse's lane schedule (debugging aid, not a test of
the kernel): the same per-lane steps, DPP moves and masks in Python, checked
against the oracle's one-read dense pass.  usage: python scripts/sim_fuse.py"""
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import oracle  # noqa: E402
from _util import SEQ_SCORES, make_read, random_seq  # noqa: E402
from rifraf_amd import RifrafSequence  # noqa: E402

NINF = -math.inf


def sim(t, r, LPT=16, fast=False, QD=4):
    m, n, bw = len(t), len(r.seq), r.bandwidth
    H = 2 * bw + abs(n - m) + 1
    c = max(m - n, 0) + bw
    vb = max(n - m, 0) + bw
    K = H + 2 * m
    assert H <= 2 * LPT - 1
    Bd = oracle.backward(t, r)          # data[d, j]
    mt, mm, ins, dl = r.match_scores, r.mismatch_scores, r.ins_scores, r.del_scores
    seq = r.seq
    out = np.full((m + 1) * 9, np.nan)
    out[:] = 12345.0                     # sentinel: every slot must be written

    def Bval(kap, d):                    # the raw load (clamped like the kernel)
        if not (0 <= d < H and 0 <= kap <= K - 1):
            return 777.0                 # garbage that must be masked
        j = (kap - d) // 2
        if j > m or j < 0:
            return 888.0
        return Bd[d, j]

    def row(ii):
        iz = min(max(ii, 0), n)
        ks = max(iz - 1, 0)
        sb = seq[max(min(ii, n), 1) - 1] if ii >= 1 else 4
        return sb, mt[ks], mm[ks], ins[ks], dl[iz]

    L = range(LPT)
    v1 = [NINF] * LPT
    v2 = [NINF] * LPT
    prev = [[NINF] * 4 for _ in L]
    accI = [[NINF] * 4 for _ in L]
    accS = [[NINF] * 4 for _ in L]
    dd = [NINF] * LPT
    R = [row(q - c) for q in L]
    kmax = K
    p = 0
    while 2 * p <= kmax:
        cb = [(t[p - q - 1] if 1 <= p - q <= m else 4) for q in L]
        for par in (0, 1):
            if par == 1:
                R = [row(q + p + 1 - c) for q in L]
            kap = 2 * p + par
            # operands per lane (before any lane updates)
            bI = [Bval(kap, 2 * q + par) if 2 * q + par < H else NINF for q in L]
            if par == 0:
                bo = [Bval(kap + 1, 2 * q + 1) if 2 * q + 1 < H and kap + 1 <= K - 1 else NINF for q in L]
                bS = [bo[q - 1] if q >= 1 else NINF for q in L]
            else:
                bS = [Bval(kap + 1, 2 * q) if 2 * q < H and kap + 1 <= K - 1 else NINF for q in L]
            E1 = [(v1[q - 1] if q >= 1 else NINF) if par == 0 else (v1[q + 1] if q + 1 < LPT else NINF) for q in L]
            nv_all = []
            for q in L:
                d = 2 * q + par
                jj = p - q
                ii = q + p + par - c
                x_ins = v1[q] if par else E1[q]
                x_del = E1[q] if par else v1[q]
                sb, rmt, rmm, ris, rds = R[q]
                ms = rmt if sb == cb[q] else rmm
                best = max(max(v2[q] + ms, x_ins + ris), x_del + rds)
                valid = d < H and 0 <= jj <= m and 0 <= ii <= n
                nv = (0.0 if (ii == 0 and jj == 0) else best) if valid else NINF
                nv_all.append(nv)
                a = jj
                jn = min(a + 1, m)
                i0 = max(0, jn - c)
                i1 = min(jn + vb, n)
                ilast = min(i1, a + vb)
                cok = 0 <= a <= m
                inrow = cok and i0 <= ii <= ilast
                peel = cok and ii == ilast + 1 and i1 > ilast
                aprev = NINF if ii < i0 else x_ins
                bSm = bS[q] if ((inrow or peel) and a < m) else NINF
                bIm = bI[q] if inrow else NINF
                dlv = nv + rds if inrow else NINF
                dsum = nv + bSm if inrow else NINF
                sub = [rmt if sb == k else rmm for k in range(4)]
                for k in range(4):
                    x = max(aprev + sub[k], prev[q][k] + ris)
                    prev[q][k] = max(x, dlv)
                    accI[q][k] = max(accI[q][k], prev[q][k] + bIm)
                    accS[q][k] = max(accS[q][k], prev[q][k] + bSm)
                dd[q] = max(dd[q], dsum)
            for q in L:
                v2[q] = v1[q]
                v1[q] = nv_all[q]
        # after the odd step: lane H >> 1 holds a finished chain (raw maxima;
        # k_reduce<true> maps -Inf to NaN outside the deletion slot)
        q = H >> 1
        a = p - q
        if 0 <= a <= m:
            base = a * 9
            for k in range(4):
                out[base + 5 + k] = math.nan if accI[q][k] == NINF else accI[q][k]
            if a < m:
                for k in range(4):
                    out[base + 9 + k] = math.nan if accS[q][k] == NINF else accS[q][k]
                out[base + 13] = dd[q]
            if a == 0:
                out[0:5] = math.nan
        # shift chain state up one lane
        prev = [[NINF] * 4] + [list(x) for x in prev[:-1]]
        accI = [[NINF] * 4] + [list(x) for x in accI[:-1]]
        accS = [[NINF] * 4] + [list(x) for x in accS[:-1]]
        dd = [NINF] + dd[:-1]
        p += 1
    return out.reshape(m + 1, 9)


def check(t, r, LPT=16):
    got = sim(t, r, LPT)
    exp, _ = oracle.cpu_pass(t, [r], nthreads=1)
    mask = np.ones_like(exp, bool)
    mask[0, :5] = False                       # not proposals (the tests' mask)
    for j in range(1, len(t) + 1):
        mask[j, t[j - 1]] = False
    eq = (got == exp) | (np.isnan(got) & np.isnan(exp)) | ~mask
    ok = bool(eq.all())
    if not ok:
        bad = np.argwhere(~eq)
        print("mismatch", len(bad), "first", bad[:6].tolist())
        for i, k in bad[:6]:
            print(i, k, got[i, k], exp[i, k])
    return ok


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    for trial in range(12):
        m = int(rng.integers(5, 40))
        t = random_seq(m, rng)
        bw = int(rng.integers(1, 6))
        r = make_read(t, rng, 0.05, bw)
        H = 2 * bw + abs(len(r.seq) - m) + 1
        if H > 31:
            continue
        print(trial, "m", m, "n", len(r.seq), "bw", bw, "H", H, check(t, r))
