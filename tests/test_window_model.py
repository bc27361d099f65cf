"""CPU model of k_sim's windowed netem/HTB resolution against the sequential
recurrence it replaces (oracle/tgoracle.c `enqueue` + `htb_until`; the kernel's netem_enqueue ->
HTB order).

The windowed algorithm is restated in plain Python at the level of the kernel's decisions
(optimistic service of the queue head, departure prefixes, the saturating occupancy counter, the
beta bound that ends a window, commit + merge); the sequential model admits, serves and releases one
candidate at a time.  Random sources cover zero and long latency, jitter > latency, heavy reorder,
duplicates (clone first), bursts and small netem limits.  This pins the algorithm; the HIP kernel
itself is checked bit for bit against the oracle by the `-m gpu` parity tests."""
import random

import pytest


def _key(it):
    e, seq, clone, _ = it
    return (e, seq, 0 if clone else 1)  # (e, seq, clone first)


class _Queue:
    def __init__(self, limit, burst, cost):
        self.ring, self.q, self.tat, self.out = [], [], 0, []
        self.limit, self.burst, self.cost = limit, burst, cost

    def serve(self, h):  # htb_until: HTB serves every item eligible before h, in key order
        self.q.sort(key=_key)
        while self.q and self.q[0][0] < h:
            e, seq, clone, ln = self.q.pop(0)
            d = max(e, self.tat)
            self.tat = max(self.tat, max(e - self.burst, 0)) + self.cost(ln)
            self.ring.append(d)
            self.out.append((d, seq, clone))

    def admit(self, T, e, seq, clone, ln):  # sequential netem_enqueue from the limit check on
        self.serve(T)
        while self.ring and self.ring[0] < T:
            self.ring.pop(0)
        if len(self.ring) + len(self.q) >= self.limit:
            return "F"
        self.q.append((e, seq, clone, ln))
        return "S"


def run_sequential(pk, limit, burst, cost, horizon):
    s = _Queue(limit, burst, cost)
    v = []
    for (T, seq, ln, cst, ec, eo) in pk:
        cv = "-" if cst == 0 else ("L" if cst == 1 else s.admit(T, ec, seq, True, ln))
        v.append(cv + s.admit(T, eo, seq, False, ln))
    s.serve(horizon)
    return v, s.out, s.ring, sorted(s.q, key=_key), s.tat


def run_windowed(pk, limit, burst, cost, horizon, W):
    s = _Queue(limit, burst, cost)
    v = [None] * len(pk)
    for b0 in range(0, len(pk), W):  # a batch = one wavefront of W lanes
        pend = list(range(b0, min(b0 + W, len(pk))))
        while pend:
            w0, T_last = pend[0], pk[pend[-1]][0]
            s.q.sort(key=_key)
            # (1) optimistic service of the queue head (at most W items)
            S = [it for it in s.q[:W] if it[0] < T_last]
            T_cut = s.q[W][0] if len(S) == W and len(s.q) > W and s.q[W][0] < T_last else None
            tat, dS, tatS = s.tat, [], []
            for (e, seq, clone, ln) in S:
                dS.append(max(e, tat))
                tat = max(tat, max(e - burst, 0)) + cost(ln)
                tatS.append(tat)
            inw = [j for j in pend if T_cut is None or pk[j][0] <= T_cut]
            # (2) departures: prefix of ring ++ served with d < T_j
            dep = s.ring + dS
            D = {}
            for j in inw:
                n = 0
                while n < len(dep) and dep[n] < pk[j][0]:
                    n += 1
                D[j] = n
            # (3) saturating occupancy counter
            x, prevD, dec = len(s.ring) + len(s.q), 0, {}
            for j in inw:
                cst = pk[j][3]
                y = x - (D[j] - prevD)
                prevD = D[j]
                dec[j] = (cst == 2 and y < limit, y + (1 if cst == 2 else 0) < limit)
                x = min(y + (2 if cst == 2 else 1), limit)
            # (4) window end: beta bound of admitted items
            wend, bmin = None, None
            for j in inw:
                if bmin is not None and bmin < pk[j][0]:
                    wend = j
                    break
                ca, oa = dec[j]
                es = [e for e, a in ((pk[j][4], ca), (pk[j][5], oa)) if a]
                if es:
                    ei = min(es)
                    pe = sum(1 for it in S if it[0] < ei)
                    b1 = dS[pe] if pe < len(S) else float("inf")
                    tb = s.tat if pe == 0 else tatS[pe - 1]
                    bi = min(b1, max(ei, tb))
                    bmin = bi if bmin is None else min(bmin, bi)
            win = [j for j in inw if wend is None or j < wend]
            # (5) commit, release, merge
            if win:
                T_w, Dw = pk[win[-1]][0], D[win[-1]]
                new_e = [e for j in win for e, a in ((pk[j][4], dec[j][0]), (pk[j][5], dec[j][1])) if a]
                e_new = min(new_e) if new_e else float("inf")
            else:
                T_w, Dw, e_new = pk[w0][0], 0, float("inf")
            nC = sum(1 for it in S if it[0] < min(e_new, T_w))
            for k in range(nC):
                it = s.q.pop(0)
                s.ring.append(dS[k])
                s.out.append((dS[k], it[1], it[2]))
            if nC:
                s.tat = tatS[nC - 1]
            del s.ring[:Dw]
            for j in win:
                T, seq, ln, cst, ec, eo = pk[j]
                ca, oa = dec[j]
                v[j] = ("-" if cst == 0 else "L" if cst == 1 else ("S" if ca else "F")) + ("S" if oa else "F")
                if oa:
                    s.q.append((eo, seq, False, ln))
                if ca:
                    s.q.append((ec, seq, True, ln))
            s.q.sort(key=_key)
            if e_new < T_w:
                s.serve(T_w)
            pend = [j for j in pend if (not win) or j > win[-1]]
    s.serve(horizon)
    return v, s.out, s.ring, sorted(s.q, key=_key), s.tat


def _source(rng, n):
    """Offered candidates of one source: (T, seq, len, clone state, clone e, original e)."""
    L, sig = rng.choice([0, 5, 50]), rng.choice([0, 3, 40])
    reo, dup = rng.choice([0, 0.1, 0.5]), rng.choice([0, 0.2])

    def e_of(T):
        if rng.random() < reo:
            return T
        return T + (max(0, L - sig + rng.randrange(2 * sig)) if sig else L)

    pk, T = [], 0
    for i in range(n):
        T += rng.choice([0, 0, 1, 2, 5])
        cst, ec = 0, None
        if rng.random() < dup:
            cst = rng.choice([1, 2])
            if cst == 2:
                ec = e_of(T)
        pk.append((T, i, rng.randrange(1, 20), cst, ec, e_of(T)))
    return pk


@pytest.mark.parametrize("W", [4, 8, 16])
def test_windowed_resolution_equals_sequential(W):
    for seed in range(1500):
        rng = random.Random(seed * 31 + W)
        limit, burst, c = rng.choice([3, 8, 20, 60]), rng.choice([0, 10, 100, 1000]), rng.choice([1, 3, 7, 20])
        pk = _source(rng, rng.randrange(1, 150))
        horizon = pk[-1][0] + rng.randrange(0, 30)
        args = (pk, limit, burst, lambda ln, c=c: ln * c // 4, horizon)
        assert run_windowed(*args, W) == run_sequential(*args), f"seed {seed}"
