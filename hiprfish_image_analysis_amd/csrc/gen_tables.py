"""Generate csrc/lp_tables.inc: compile-time constants for the fused enhancement kernels.

* LP2D_11_9[9][11][2], LP3D_11_9_9[72][11][3]: line-profile sampling offsets for the
  reference's fixed parameters (neighbor2d.pyx:32-55 with patch 11 / phi 9; neighbor.pyx
  :209-243 with patch 11 / theta 9 / phi 9); LP3D_V3_11_9_9 the variant table of
  line_profile_memory_efficient_v3 (neighbor.pyx:293-311).  Computed by an independent restatement of
  the table construction; tests/test_tables.py checks them against the reference-derived
  golden tables and against hrf_lp_table_2d/3d.
* SEL9 / SEL72: comparator lists of Knuth's merge-exchange sort (TAOCP 5.2.2 Algorithm M)
  pruned backwards to the order statistics the enhancement needs (ranks 2, 3, 6 and 7 of
  9 values; ranks 17, 18, 53 and 54 of 72 values).

Run: python csrc/gen_tables.py  (rewrites lp_tables.inc next to this file)
"""
import math
import os
import random


def sample_line(patch, iv):
    inc = (patch - 1) // 2
    ndim = len(iv)
    arg = max(range(ndim), key=lambda k: (abs(iv[k]), -k))
    line_n = 2 * abs(iv[arg]) + 1
    base = (patch - line_n) // 2 if line_n < patch else 0
    off = [[0] * ndim for _ in range(patch)]
    for li in range(line_n):
        for k in range(ndim):
            s = (iv[k] > 0) - (iv[k] < 0)
            h = float(s * li) * float(2 * abs(iv[k]) + 1) / float(line_n)
            tr = math.copysign(math.floor(abs(h)), h) if h != 0 else 0.0
            off[li + base][k] = int(tr + inc - iv[k])
    if line_n < patch:
        for li in range(base):
            off[li] = list(off[base])
            off[li + line_n + base] = list(off[line_n + base - 1])
    return off


def table_2d(patch=11, nphi=9):
    inc = (patch - 1) // 2
    out = []
    for phi in range(nphi):
        a = phi * math.pi / nphi
        out.append(sample_line(patch, [round(inc * math.cos(a)), round(inc * math.sin(a))]))
    return out


def table_3d(patch=11, ntheta=9, nphi=9):
    inc = (patch - 1) // 2
    out = []
    for th in range(1, ntheta):
        for phi in range(nphi):
            ap = phi * math.pi / nphi
            at = th * math.pi / ntheta
            out.append(sample_line(patch, [round(inc * math.cos(ap) * math.sin(at)),
                                           round(inc * math.sin(ap) * math.sin(at)),
                                           round(inc * math.cos(at))]))
    return out


def sample_line_v3(patch, iv):
    """neighbor.pyx:293-311 (line_profile_memory_efficient_v3): like sample_line but
    np.round on the short-line branch and np.floor of s*li*(2*iv+1)/line_n (signed iv) on
    the full-length one"""
    inc = (patch - 1) // 2
    ndim = len(iv)
    arg = max(range(ndim), key=lambda k: (abs(iv[k]), -k))
    line_n = 2 * abs(iv[arg]) + 1
    off = [[0] * ndim for _ in range(patch)]
    if line_n < patch:
        base = (patch - line_n) // 2
        for li in range(line_n):
            for k in range(ndim):
                s = (iv[k] > 0) - (iv[k] < 0)
                h = float(s * li) * float(2 * abs(iv[k]) + 1) / float(line_n)
                off[li + base][k] = int(round(h) + inc - iv[k])
        for li in range(base):
            off[li] = list(off[base])
            off[li + line_n + base] = list(off[line_n + base - 1])
    else:
        for li in range(line_n):
            for k in range(ndim):
                s = (iv[k] > 0) - (iv[k] < 0)
                h = float(s * li) * float(2 * iv[k] + 1) / float(line_n)
                off[li][k] = int(math.floor(h) + inc - iv[k])
    return off


def table_3d_v3(patch=11, ntheta=9, nphi=9):
    inc = (patch - 1) // 2
    out = []
    for th in range(1, ntheta):
        for phi in range(nphi):
            ap = phi * math.pi / nphi
            at = th * math.pi / ntheta
            out.append(sample_line_v3(patch, [round(inc * math.cos(ap) * math.sin(at)),
                                              round(inc * math.sin(ap) * math.sin(at)),
                                              round(inc * math.cos(at))]))
    return out


def merge_exchange(n):
    """Knuth Algorithm M: comparator list sorting any n inputs ascending."""
    comps = []
    t = max(1, math.ceil(math.log2(n)))
    p = 1 << (t - 1)
    while p > 0:
        q, r, d = 1 << (t - 1), 0, p
        while True:
            for i in range(n - d):
                if (i & p) == r:
                    comps.append((i, i + d))
            if q == p:
                break
            d, q, r = q - p, q >> 1, p
        p >>= 1
    return comps


def prune(comps, outputs):
    need = set(outputs)
    kept = []
    for a, b in reversed(comps):
        if a in need or b in need:
            kept.append((a, b))
            need.add(a)
            need.add(b)
    return list(reversed(kept))


def check(comps, n, outputs, trials=3000):
    rng = random.Random(7)
    for _ in range(trials):
        v = [rng.choice([rng.random(), float(rng.randint(0, 3))]) for _ in range(n)]
        w = list(v)
        for a, b in comps:
            if w[a] > w[b]:
                w[a], w[b] = w[b], w[a]
        s = sorted(v)
        assert all(w[o] == s[o] for o in outputs), "selection network broken"


def main():
    t2 = table_2d()
    t3 = table_3d()
    t3v3 = table_3d_v3()
    sel9 = prune(merge_exchange(9), [2, 3, 6, 7])
    sel72 = prune(merge_exchange(72), [17, 18, 53, 54])
    check(sel9, 9, [2, 3, 6, 7])
    check(sel72, 72, [17, 18, 53, 54])
    lines = ["// Generated by gen_tables.py -- do not edit.", "#pragma once", "#include <cstdint>", ""]
    lines.append("constexpr int8_t LP2D_11_9[9][11][2] = {")
    for d in t2:
        lines.append("  {" + ", ".join("{%d, %d}" % tuple(o) for o in d) + "},")
    lines.append("};")
    for name, tab in [("LP3D_11_9_9", t3), ("LP3D_V3_11_9_9", t3v3)]:
        lines.append("constexpr int8_t %s[72][11][3] = {" % name)
        for d in tab:
            lines.append("  {" + ", ".join("{%d, %d, %d}" % tuple(o) for o in d) + "},")
        lines.append("};")
    for name, sel in [("SEL9", sel9), ("SEL72", sel72)]:
        lines.append("constexpr int %s_N = %d;" % (name, len(sel)))
        lines.append("constexpr uint8_t %s[%d][2] = {" % (name, len(sel)))
        for i in range(0, len(sel), 12):
            lines.append("  " + " ".join("{%d, %d}," % c for c in sel[i:i + 12]))
        lines.append("};")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lp_tables.inc")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("wrote", path, "sel9", len(sel9), "sel72", len(sel72))


if __name__ == "__main__":
    main()
