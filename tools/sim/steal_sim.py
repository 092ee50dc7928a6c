"""Event simulation of the frontier kernel's per-SIMD timeline from a heavy_g*.npz
(tools/mb_heavy_predict.py): each wave's slots, its SIMD.  Model: a wave on a
SIMD with n resident walking waves spends L(n) = max(SOLO, n * THR) us per slot.
Variants: as measured (placement from HW_ID), and work stealing (a wave that
ends takes half of the remaining slots of the heaviest walk still running whose
remainder is above MIN, after a hand-off delay)."""
import sys
import heapq
import numpy as np

SOLO, THR = 3.0, 1.14


def simd_of(hw):
    hid = hw[:, 0].astype(np.int64); x = hw[:, 1].astype(np.int64)
    return ((hid >> 4) & 3) | (((hid >> 8) & 15) << 2) | (((hid >> 12) & 1) << 6) | (((hid >> 13) & 7) << 7) | (x << 10)


def simulate(slots, simd, steal=False, min_rem=30, delay=5.0, dt=1.0):
    # time-stepped: each wave has remaining slots; per step dt, progress dt / L(n_simd)
    waves = [dict(rem=float(s), simd=int(m), end=None) for s, m in zip(slots, simd)]
    t = 0.0
    while True:
        active = [w for w in waves if w["end"] is None and w["rem"] > 0]
        if not active:
            break
        cnt = {}
        for w in active:
            cnt[w["simd"]] = cnt.get(w["simd"], 0) + 1
        for w in active:
            w["rem"] -= dt / max(SOLO, cnt[w["simd"]] * THR)
        t += dt
        for w in active:
            if w["rem"] <= 0:
                w["end"] = t
                if steal:
                    # the freed wave slot steals half of the heaviest remaining walk
                    cand = [v for v in waves if v["end"] is None and v["rem"] > min_rem]
                    if cand:
                        v = max(cand, key=lambda v: v["rem"])
                        half = v["rem"] / 2
                        v["rem"] -= half
                        waves.append(dict(rem=half + delay / SOLO, simd=w["simd"], end=None))
    return t


if __name__ == "__main__":
    for g in sys.argv[1:]:
        d = np.load(g)
        h = d["stamps"].astype(np.int64)
        sl = h[:, 2].astype(float)
        sm = simd_of(d["hwid"])
        span = (h[:, 1].max() - h[:, 0].min()) / 100
        print(g, f"measured {span:.0f} us; model {simulate(sl, sm):.0f}; steal {simulate(sl, sm, True):.0f}; "
              f"steal min60 {simulate(sl, sm, True, 60):.0f}")
