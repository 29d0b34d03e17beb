"""Generate the constant tables of hrf_cr_log / hrf_cr_log10 (detmath.h) with Python's decimal
module: ln(k/128) for k = 96..192 as double-double (hi, lo) pairs, ln 2, 1/3, 1/5 and 1/ln 10 as
double-doubles.  Rewrites the block between the BEGIN/END LOGTAB markers of detmath.h.

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
    open(path, "w").write(src[:a] + "\n".join(out) + src[b:])
    print("wrote", path)


if __name__ == "__main__":
    main()
