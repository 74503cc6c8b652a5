"""The schedule of band_lane2_kernel (csrc/ovl_dp_lane.hip), emulated on the CPU: a pair's band cells split over
two lanes, lane 1 one row behind lane 0, the carries between them (lane 0's last cell of the previous row as lane
1's left, lane 1's first new cell as lane 0's last up, lane 1's bottom window code as lane 0's new top code), the
virtual leading rows, the extra last step and the two scans -- step for step as the kernel orders them, against
oracle.banded_py (the band knob's statement).  The GPU tests (test_gpu_banded.py, OVL_BAND_FORM=lane2) check the
kernel itself; this pins the schedule on the CPU."""
import random

import pytest


def _lane2(oracle_mod, s, t, match, mismatch, indel, W):
    NB = 2 * W + 1
    H = (NB + 1) // 2
    NEG, PAD = -(1 << 30), 4
    code = {"A": 0, "C": 1, "G": 2, "T": 3}
    n, m = len(s), len(t)
    _, jstar = oracle_mod.ungapped(s, t, match, mismatch)
    g = indel
    s_ma, s_mm, s_pad, s_virt = match - 2 * g, mismatch - 2 * g, -2 * g, -g
    cc = n - jstar + W
    R = (n + 3) // 4 * 4  # one pair per wavefront: nmax = n
    sk = R - n
    u0, ub = -sk - cc, NB - sk - cc

    def tcode(u):
        return PAD if u < 0 else code[t[min(u, m - 1)]]

    def scode(it):
        return code[s[min(max(it - sk, 0), n - 1)]]

    lanes = []
    for h in (0, 1):
        kbase = H - 1 if h else -1  # lane 0: diagonals -1 (dummy) .. H-2; lane 1: H-1 .. NB-1
        uw = u0 - h + kbase          # lane h starts before iteration -h
        V = [-g * (uw + j) for j in range(H)]
        if not h:
            V[0] = NEG
        lanes.append({"kbase": kbase, "T": [tcode(uw + j) for j in range(H)], "V": V})
    prev = [0, tcode(ub - 1)]  # row symbol / entering code of the previous step's iteration (-1 before step 0)

    def step(t_step, x_c, tn_c):
        x = {0: x_c, 1: prev[0]}
        tn = {0: tn_c, 1: prev[1]}
        prev[:] = [x_c, tn_c]
        left = {0: NEG, 1: lanes[0]["V"][H - 1]}  # swap at the step's start
        upin = {0: NEG, 1: NEG}
        for j in range(H):
            vals = {}
            for h in (0, 1):
                L = lanes[h]
                if t_step - h < sk:
                    s2 = s_virt
                else:
                    tc = L["T"][j]
                    s2 = s_pad if tc >= 4 else (s_ma if tc == x[h] else s_mm)
                up = L["V"][j + 1] if j + 1 < H else upin[h]
                v = max(L["V"][j] + s2, up, left[h])
                vals[h] = NEG if (j == 0 and h == 0) else v
            if j == 0:
                upin[0] = vals[1]  # lane 1's first cell, just computed, is lane 0's last up
            for h in (0, 1):
                lanes[h]["V"][j] = left[h] = vals[h]
        for L in lanes:
            L["T"] = L["T"][1:] + [0]
        lanes[0]["T"][H - 1] = lanes[1]["T"][0]
        lanes[1]["T"][H - 1] = tn[1]

    for t_step in range(R):
        step(t_step, scode(t_step), tcode(t_step + ub))
    v0 = list(lanes[0]["V"])  # lane 0 is done after iteration R - 1
    step(R, 0, 0)             # lane 1's last iteration
    best, bend = -(1 << 31), -1
    for h, V in ((0, v0), (1, lanes[1]["V"])):
        for jl in range(1 if h == 0 else 0, H):
            j = jstar - W + lanes[h]["kbase"] + jl
            v = V[jl] + g * (n + j)
            if 0 <= j <= m and v > best:
                best, bend = v, j
    return best, bend


@pytest.mark.parametrize("W", [1, 2, 3, 5, 8, 24, 40])
def test_two_lane_schedule_matches_banded_oracle(oracle_mod, W):
    rng = random.Random(W)
    for _ in range(60):
        n, m = rng.randint(1, 60), rng.randint(1, 60)
        s = "".join(rng.choice("ACGT") for _ in range(n))
        t = "".join(rng.choice("ACGT") for _ in range(m))
        if rng.random() < 0.5 and n > 3:  # an overlap: t continues a suffix of s
            k = rng.randint(1, n - 1)
            t = (s[k:] + t)[:m]
        params = rng.choice([(10, -1, -2), (1, -1, -1), (2, -3, -5), (5, -4, -1), (3, 2, -1), (10, -1, -30)])
        assert _lane2(oracle_mod, s, t, *params, W) == tuple(oracle_mod.banded_py(s, t, *params, W)), (s, t, params)
