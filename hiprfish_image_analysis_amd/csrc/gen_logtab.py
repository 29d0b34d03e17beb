"""Generate the constant tables of hrf_cr_log / hrf_cr_log10 (detmath.h) with Python's decimal
module: ln(k/128) for k = 96..192 as double-double (hi, lo) pairs, ln 2, 1/3, 1/5 and 1/ln 10 as
double-doubles; 2^(j/64) for j = 0..63 (hrf_exp_neg_tab, the NL-means weights).  Rewrites the
blocks between the BEGIN/END LOGTAB and BEGIN/END EXPTAB markers of detmath.h.

Run: python csrc/gen_logtab.py
"""
import decimal
import os

decimal.getcontext().prec = 80
D = decimal.Decimal


def dd(v):
    hi = float(v)
    lo = float(v - D(hi))
    return hi, lo


def main():
    rows = []
    for k in range(96, 193):
        rows.append(dd((D(k) / D(128)).ln()))
    ln2 = dd(D(2).ln())
    third = dd(D(1) / D(3))
    fifth = dd(D(1) / D(5))
    il10 = dd(D(1) / D(10).ln())
    out = ["/* BEGIN LOGTAB (gen_logtab.py) */",
           "HRF_DM_TAB double hrf_logtab_hi[97] = {"]
    out += ["  %s," % ", ".join(repr(h) for h, _ in rows[i:i + 4]) for i in range(0, 97, 4)]
    out += ["};", "HRF_DM_TAB double hrf_logtab_lo[97] = {"]
    out += ["  %s," % ", ".join(repr(l) for _, l in rows[i:i + 4]) for i in range(0, 97, 4)]
    out += ["};"]
    for name, (h, l) in (("LN2", ln2), ("THIRD", third), ("FIFTH", fifth), ("INVLN10", il10)):
        out.append("#define HRF_DD_%s_HI %s" % (name, repr(h)))
        out.append("#define HRF_DD_%s_LO %s" % (name, repr(l)))
    out.append("/* END LOGTAB */")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "detmath.h")
    src = open(path).read()
    a = src.index("/* BEGIN LOGTAB")
    b = src.index("/* END LOGTAB */") + len("/* END LOGTAB */")
    src = src[:a] + "\n".join(out) + src[b:]
    e = [float(D(2) ** (D(j) / D(64))) for j in range(64)]
    inv = float(D(64) / D(2).ln())
    l2 = D(2).ln() / D(64)
    l2hi = float(l2)
    l2lo = float(l2 - D(l2hi))
    out = ["/* BEGIN EXPTAB (gen_logtab.py) */", "HRF_DM_TAB double hrf_exp2tab64[64] = {"]
    out += ["  %s," % ", ".join(repr(v) for v in e[i:i + 4]) for i in range(0, 64, 4)]
    out += ["};", "#define HRF_EXP_INVL %s" % repr(inv), "#define HRF_EXP_L2HI %s" % repr(l2hi),
            "#define HRF_EXP_L2LO %s" % repr(l2lo), "/* END EXPTAB */"]
    a = src.index("/* BEGIN EXPTAB")
    b = src.index("/* END EXPTAB */") + len("/* END EXPTAB */")
    open(path, "w").write(src[:a] + "\n".join(out) + src[b:])
    print("wrote", path)


if __name__ == "__main__":
    main()
