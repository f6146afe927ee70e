"""Generate tests/golden/serialstep.json: the reference's SERIALIZABLE
known-answer tests (tests/serialstep.test, driven by tests/tools/stepper.c)
restated as read sets + write sets at the level the check sees them.

Run in the build container (it reads the expected outputs from
/root/reference to record the failure counts; the committed JSON is all the
tests need):   python tests/golden/make_serialstep.py

Restatement rules (how the SQL of each scenario becomes CurRange's and logged
keys; db/sqlglue.c cursor capture, bdb/ll.c logging):
  * a point lookup on a unique index -> range [k, k] on that index;
  * `where id < v` -> range (open, k(v)]; `where id > v` -> [k(v), open);
    `id >= a and id <= b` -> [k(a), k(b+1)] (the cursor stops on the next row);
  * `where col = 'x'` on a dup index -> prefix range [k(x), k(x)] (the dup key
    carries a genid suffix, so the 9-byte endpoint is a prefix, s9);
  * a full scan (`select * ... order by id`, or an update without where)
    touches both ends -> islocked range on the table (db/sqlglue.c:3903-3904);
  * an update of non-key columns logs upd_dta + upd_ix of every index key of
    the row (unchanged keys are re-logged with the new genid, bdb/ll.c:749);
    a key change logs del_ix(old) + add_ix(new); insert add_dta + add_ix;
    delete del_dta + del_ix;
  * read-only transactions never ship a read set (db/sqloffload.c:280-287).
Index keys follow db/types.c:766-771 (0x08 + big-endian, sign bit flipped);
intervals (s15), datetimes (s7) and decimals (s8) use order-preserving int64
stand-ins (the check compares key bytes only).
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from comdb2_amd import formats as F  # noqa: E402

REF = "/root/reference/tests/serialstep.test"

USERS = {  # id: (name, age) -- the s1-s6 setup rows (sN_01.req, session 5)
    1: ("aaa", 18), 2: ("dsa", 40), 3: ("afd", 65), 6: ("bda", 23), 4: ("rte", 34),
    5: ("anh", 21), 9: ("try", 20), 7: ("aer", 56), 8: ("jyf", 33), 99: ("ytu", 8),
    10: ("htr", 54)}


def users_keys(uid, name, age, genid):
    """users.csc2: KEY_ID = id; dup KEY_AGE = age + id; dup KEY_NAME = name."""
    return {0: F.enc_int64(uid),
            1: F.enc_int64(age) + F.enc_int64(uid) + F.enc_genid(genid),
            2: F.enc_cstring(name, 30) + F.enc_genid(genid)}


def dots_keys(did, color, genid):
    """dots.csc2: KEY_ID = id; dup KEY_COLOR = color (cstring[8])."""
    return {0: F.enc_int64(did), 1: F.enc_cstring(color, 8) + F.enc_genid(genid)}


def upd_same(tb, keys):
    w = [("upd_dta", tb, -2, None)]
    return w + [("upd_ix", tb, ix, k.hex()) for ix, k in sorted(keys.items())]


def ins(tb, keys):
    return [("add_dta", tb, -2, None)] + [("add_ix", tb, ix, k.hex()) for ix, k in sorted(keys.items())]


def dele(tb, keys):
    return [("del_dta", tb, -2, None)] + [("del_ix", tb, ix, k.hex()) for ix, k in sorted(keys.items())]


def rng_(tb, ix, lo=None, hi=None, lflag=0, rflag=0, locked=0):
    return dict(tb=tb, ix=ix, lkey=None if lo is None else lo.hex(),
                rkey=None if hi is None else hi.hex(), lflag=lflag, rflag=rflag, islocked=locked)


def locked(tb):
    return rng_(tb, -1, lflag=1, rflag=1, locked=1)


def K(v):
    return F.enc_int64(v)


def scenarios():
    g = {u: 1000 + u for u in USERS}          # genid of each users row
    uk = {u: users_keys(u, USERS[u][0], USERS[u][1], g[u]) for u in USERS}
    ng = lambda u: 5000 + u                    # genid after an update
    out = {}

    # s1: write-skew ring, commit order 1,2,3,4 -> T2 and T4 fail
    out["s1"] = dict(
        txns={
            "T1": dict(reads=[rng_("users", 0, K(1), K(1)), rng_("users", 0, K(4), K(4))],
                       writes=upd_same("users", users_keys(4, "rte", 34, ng(4)))),
            "T2": dict(reads=[rng_("users", 0, K(4), K(4)), rng_("users", 0, K(7), K(7))],
                       writes=upd_same("users", users_keys(7, "aer", 56, ng(7)))),
            "T3": dict(reads=[rng_("users", 0, K(7), K(7)), rng_("users", 0, K(10), K(10))],
                       writes=upd_same("users", users_keys(10, "htr", 54, ng(10)))),
            "T4": dict(reads=[rng_("users", 0, K(10), K(10)), rng_("users", 0, K(1), K(1))],
                       writes=upd_same("users", users_keys(1, "aaa", 18, ng(1)))),
        },
        events=[["begin", "T1"], ["begin", "T2"], ["begin", "T3"], ["begin", "T4"],
                ["commit", "T1"], ["commit", "T2"], ["commit", "T3"], ["commit", "T4"]],
        expect_fail=["T2", "T4"])

    # s2: T2 full scan (locked) loses to T1's delete; T4 is read-only
    t2w = []
    for u in (1, 3, 5, 7, 9, 99):
        t2w += upd_same("users", users_keys(u, USERS[u][0], USERS[u][1], ng(u)))
    r88 = users_keys(88, "dasd", 88, 7088)
    out["s2"] = dict(
        txns={
            "T1": dict(reads=[rng_("users", 0, K(99), K(99))], writes=dele("users", uk[99])),
            "T2": dict(reads=[locked("users")] + [rng_("users", 0, K(u), K(u))
                                                  for u in (1, 3, 5, 7, 9, 88, 99)],
                       writes=t2w),
            "T3": dict(reads=[rng_("users", 0, K(88), K(88))],
                       writes=ins("users", r88) + dele("users", r88)),
            "T4": dict(reads=[locked("users")], writes=[]),
        },
        events=[["begin", "T1"], ["begin", "T2"], ["begin", "T3"], ["begin", "T4"],
                ["commit", "T1"], ["commit", "T2"], ["commit", "T3"], ["commit", "T4"]],
        expect_fail=["T2"])

    def s34(order):
        t1w = upd_same("users", users_keys(1, "aaa", 18, ng(1))) + \
            upd_same("users", users_keys(2, "dsa", 40, ng(2)))
        t2w = upd_same("users", users_keys(10, "htr", 54, ng(10))) + \
            upd_same("users", users_keys(99, "ytu", 8, ng(99)))
        return dict(
            txns={
                "T1": dict(reads=[locked("users"), rng_("users", 0, None, K(3), lflag=1)], writes=t1w),
                "T2": dict(reads=[rng_("users", 0, K(5), K(8)), rng_("users", 0, K(9), None, rflag=1)],
                           writes=t2w),
            },
            events=[["begin", "T1"], ["begin", "T2"]] + [["commit", t] for t in order],
            expect_fail=[] if order == ["T1", "T2"] else ["T1"])

    out["s3"] = s34(["T1", "T2"])
    out["s4"] = s34(["T2", "T1"])

    # s5: T3 reads everything after T1/T2 commit but is read-only
    out["s5"] = dict(
        txns={
            "T1": dict(reads=[rng_("users", 0, None, K(3), lflag=1)],
                       writes=upd_same("users", users_keys(1, "aaa", 18, ng(1))) +
                       upd_same("users", users_keys(2, "dsa", 40, ng(2)))),
            "T2": dict(reads=[rng_("users", 0, K(9), None, rflag=1)],
                       writes=upd_same("users", users_keys(10, "htr", 54, ng(10))) +
                       upd_same("users", users_keys(99, "ytu", 8, ng(99)))),
            "T3": dict(reads=[locked("users")], writes=[]),
        },
        events=[["begin", "T1"], ["begin", "T2"], ["begin", "T3"],
                ["commit", "T1"], ["commit", "T2"], ["commit", "T3"]],
        expect_fail=[])

    # s9: dots recolour; prefix ranges over the dup KEY_COLOR index
    dg = {d: 2000 + d for d in range(1, 11)}
    col = {d: "B" if d % 2 else "W" for d in range(1, 11)}

    def recolour(ids, new):
        w = []
        for d in ids:
            old = dots_keys(d, col[d], dg[d])
            nw = dots_keys(d, new, 9000 + d)
            w += [("upd_dta", "dots", -2, None), ("upd_ix", "dots", 0, nw[0].hex()),
                  ("del_ix", "dots", 1, old[1].hex()), ("add_ix", "dots", 1, nw[1].hex())]
        return w

    wkey = F.enc_cstring("W", 8)
    bkey = F.enc_cstring("B", 8)
    out["s9"] = dict(
        txns={
            "T1": dict(reads=[rng_("dots", 1, wkey, wkey)],
                       writes=recolour([d for d in col if col[d] == "W"], "B")),
            "T2": dict(reads=[rng_("dots", 1, bkey, bkey)],
                       writes=recolour([d for d in col if col[d] == "B"], "W")),
        },
        events=[["begin", "T1"], ["begin", "T2"], ["commit", "T2"], ["commit", "T1"]],
        expect_fail=["T1"])
    out.update(later_scenarios(uk))
    return out


def enc_int32(v):
    """One int (4-byte) field: 0x08 + big-endian(v ^ 2^31) (db/types.c)."""
    return bytes([0x08]) + ((int(v) ^ (1 << 31)) & 0xFFFFFFFF).to_bytes(4, "big")


def later_scenarios(uk):
    """s6, s10-s15.  runit has no .fastinit files, so tables persist across
    the cases, which run in glob order (s10 .. s15, s1 .. s9): s10-s15 start
    from empty tables, s6 sees the users rows left by s1-s5 (s2 deleted 99)."""
    out = {}
    ng = lambda u: 6000 + u                    # genid after s6's update

    # s6: T1 rewrites every row under a table lock and commits first; T2's
    # age-99 prefix range sees none of those keys (no row is 99 years old);
    # T3's id-88 update finds no row, so it is read-only and never checked
    t1w = []
    for u in sorted(uk):
        if u != 99:
            t1w += upd_same("users", users_keys(u, USERS[u][0], USERS[u][1], ng(u)))
    r99 = users_keys(99, "nn", 99, 7099)
    out["s6"] = dict(
        txns={
            "T1": dict(reads=[locked("users")], writes=t1w),
            "T2": dict(reads=[rng_("users", 1, K(99), K(99))], writes=ins("users", r99) + dele("users", r99)),
            "T3": dict(reads=[rng_("users", 0, K(88), K(88))], writes=[]),
        },
        events=[["begin", "T1"], ["begin", "T2"], ["begin", "T3"],
                ["commit", "T1"], ["commit", "T2"], ["commit", "T3"]],
        expect_fail=[])

    # s10: mytab (dup KEY_CLASS = class, dup KEY_VALUE = value); each txn sums
    # one class (prefix range on KEY_CLASS) and inserts into the other
    def mytab_keys(cls, val, genid):
        return {0: K(cls) + F.enc_genid(genid), 1: K(val) + F.enc_genid(genid)}

    out["s10"] = dict(
        txns={
            "T1": dict(reads=[rng_("mytab", 0, K(1), K(1))], writes=ins("mytab", mytab_keys(2, 30, 3005))),
            "T2": dict(reads=[rng_("mytab", 0, K(2), K(2))], writes=ins("mytab", mytab_keys(1, 300, 3006))),
        },
        events=[["begin", "T1"], ["begin", "T2"], ["commit", "T2"], ["commit", "T1"]],
        expect_fail=["T1"])

    # s11: colors (KEY_ID = id, dup KEY_COLOR = color), rows cycle Y, B, R.
    # The reference inserts 9000 rows; restated over the first 90 (the
    # verdicts depend only on the key order, which the cycle keeps).  A dup
    # equality scan stops on the first row past the value, so the captured
    # range ends at that row's key (B -> first R row; R -> first Y row; Y is
    # the last value: the scan runs off the end, right side open).
    ids = range(1, 91)
    colour = {i: "YBR"[(i - 1) % 3] for i in ids}
    cg = {i: 4000 + i for i in ids}
    ckey = lambda c, g: F.enc_cstring(c, 8) + F.enc_genid(g)

    def recolour_c(frm, to, gbase):
        w = []
        for i in ids:
            if colour[i] == frm:
                w += [("upd_dta", "colors", -2, None), ("upd_ix", "colors", 0, K(i).hex()),
                      ("del_ix", "colors", 1, ckey(frm, cg[i]).hex()),
                      ("add_ix", "colors", 1, ckey(to, gbase + i).hex())]
        return w

    first = {c: min(i for i in ids if colour[i] == c) for c in "YBR"}
    pre = lambda c: F.enc_cstring(c, 8)
    out["s11"] = dict(
        txns={
            "T1": dict(reads=[rng_("colors", 1, pre("R"), ckey("Y", cg[first["Y"]]))],
                       writes=recolour_c("R", "Y", 10000)),
            "T2": dict(reads=[rng_("colors", 1, pre("Y"), None, rflag=1)],
                       writes=recolour_c("Y", "B", 20000)),
            "T3": dict(reads=[rng_("colors", 1, pre("B"), ckey("R", cg[first["R"]]))],
                       writes=recolour_c("B", "R", 30000)),
        },
        events=[["begin", "T1"], ["begin", "T2"], ["begin", "T3"],
                ["commit", "T1"], ["commit", "T2"], ["commit", "T3"]],
        expect_fail=["T2", "T3"])

    # s12: control (KEY_DN = deposit_no) holds one row; the sub-select and the
    # select scan the whole table (table lock); T2 moves the row's key 1 -> 2
    out["s12"] = dict(
        txns={
            "T1": dict(reads=[locked("control")],
                       writes=ins("receipt", {0: K(4), 1: K(1) + F.enc_genid(5004)})),
            "T2": dict(reads=[locked("control")],
                       writes=[("upd_dta", "control", -2, None), ("del_ix", "control", 0, K(1).hex()),
                               ("add_ix", "control", 0, K(2).hex())]),
        },
        events=[["begin", "T1"], ["begin", "T2"], ["commit", "T2"], ["commit", "T1"]],
        expect_fail=["T1"])

    # s13: rollover (KEY_ID = id); T1 reads row 2 and updates row 1, T2
    # updates row 2 and commits first
    out["s13"] = dict(
        txns={
            "T1": dict(reads=[rng_("rollover", 0, K(2), K(2)), rng_("rollover", 0, K(1), K(1))],
                       writes=upd_same("rollover", {0: K(1)})),
            "T2": dict(reads=[rng_("rollover", 0, K(2), K(2))], writes=upd_same("rollover", {0: K(2)})),
        },
        events=[["begin", "T1"], ["begin", "T2"], ["commit", "T2"], ["commit", "T1"]],
        expect_fail=["T1"])

    # s14: t1 (ID = int id); an autocommit update (A1, not serializable, so
    # its own check never fires) moves id 1 -> 11 while T2 has read id 1
    mv = lambda a, b: [("upd_dta", "t1", -2, None), ("del_ix", "t1", 0, enc_int32(a).hex()),
                       ("add_ix", "t1", 0, enc_int32(b).hex())]
    out["s14"] = dict(
        txns={
            "T2": dict(reads=[rng_("t1", 0, enc_int32(1), enc_int32(1))], writes=mv(1, 2)),
            "A1": dict(reads=[rng_("t1", 0, enc_int32(1), enc_int32(1))], writes=mv(1, 11)),
        },
        events=[["begin", "T2"], ["begin", "A1"], ["commit", "A1"], ["commit", "T2"]],
        expect_fail=["T2"])

    # s15: intv (KEY_ID = id, dup KEY_YM = intervalym, dup KEY_DS =
    # intervalds), two rounds of the s3-style skew, once over each interval
    # index.  Stand-in key encoding: the interval as an int64 count of months /
    # milliseconds in the A9 int64 format (order-preserving, which is all the
    # byte comparisons of the check see); not comdb2's interval on-disk format.
    ym = {i: 13 * i for i in range(1, 6)}                       # '01-01' .. '05-05'
    ds = {i: ((i * 24 + i) * 3600 + i * 61) * 1000 + 10 * i for i in range(1, 6)}

    def intv_keys(i, g):
        return {0: K(i), 1: K(ym[i]) + F.enc_genid(g), 2: K(ds[i]) + F.enc_genid(g)}

    def upd_rows(ids, g):
        w = []
        for i in ids:
            w += upd_same("intv", intv_keys(i, g + i))
        return w

    ym_lo, ym_hi = 2 * 12 + 10, 4 * 12                         # '02-10', '04-00'
    ds_lo, ds_hi = (2 * 24 + 10) * 3600 * 1000, 4 * 24 * 3600 * 1000
    out["s15"] = dict(
        txns={
            "T1a": dict(reads=[rng_("intv", 1, None, K(ym_lo), lflag=1)], writes=upd_rows((4, 5), 8100)),
            "T2a": dict(reads=[rng_("intv", 1, K(ym_hi), None, rflag=1)], writes=upd_rows((1, 2), 8150)),
            "T1b": dict(reads=[rng_("intv", 2, None, K(ds_lo), lflag=1)], writes=upd_rows((4, 5), 8200)),
            "T2b": dict(reads=[rng_("intv", 2, K(ds_hi), None, rflag=1)], writes=upd_rows((1, 2), 8250)),
        },
        events=[["begin", "T1a"], ["begin", "T2a"], ["commit", "T1a"], ["commit", "T2a"],
                ["begin", "T1b"], ["begin", "T2b"], ["commit", "T1b"], ["commit", "T2b"]],
        expect_fail=["T2a", "T2b"])
    out.update(shows_scenarios())
    return out


def shows_scenarios():
    """s7 / s8 on shows (shows.csc2: KEY_ID = id, dup KEY_DATE = date
    (datetime), dup KEY_DEC = dec (decimal128)).  Both run on the 7 rows the
    s7 setup inserts (s8 runs after s7 in glob order; tables persist).
    Stand-in key encodings, order-preserving, which is all the byte
    comparisons of the check see (as for s15's intervals): a datetime is its
    UTC instant in milliseconds, a decimal its value x 10^4 (every value has at
    most 4 decimals), both in the A9 int64 format; not comdb2's on-disk
    datetime / decimal128 formats.  Session time zone America/New_York
    (comdb2's default) for the literals without one; the UTC offsets of the
    dates' zones on those days are spelled out below."""
    import datetime as dt

    def utc_ms(y, mo, d, h, mi, se, off_h):
        t = dt.datetime(y, mo, d, h, mi, se, tzinfo=dt.timezone(dt.timedelta(hours=off_h)))
        return int(t.timestamp() * 1000)

    rows = {  # id: (date ms, dec x 1e4) -- s7_01.req, session 1
        1: (utc_ms(2014, 10, 8, 16, 0, 8, -4), 12131),    # America/New_York, EDT
        2: (utc_ms(2014, 12, 21, 14, 35, 0, -5), 2149),   # session zone, EST
        3: (utc_ms(2014, 12, 21, 14, 35, 0, 8), 34320),   # Asia/Shanghai
        7: (utc_ms(2011, 3, 26, 13, 12, 47, 8), 10000),   # Asia/Hong_Kong
        12: (utc_ms(2014, 9, 28, 14, 35, 0, -4), 65443),  # America/Toronto, EDT
        8: (utc_ms(2014, 5, 1, 0, 0, 0, 8), 82443),       # Asia/Taipei
        10: (utc_ms(2014, 1, 1, 0, 0, 0, -8), 23210),     # US/Pacific, PST
    }

    def keys(i, genid):
        d, m = rows[i]
        return {0: K(i), 1: K(d) + F.enc_genid(genid), 2: K(m) + F.enc_genid(genid)}

    def upd(ids, g):
        w = []
        for i in ids:
            w += upd_same("shows", keys(i, g + i))
        return w

    late = utc_ms(2014, 10, 8, 17, 0, 0, -4)    # '2014-10-08T17:00:00 America/New_York'
    early = utc_ms(2014, 1, 1, 0, 0, 0, -5)     # '2014-01-01T00:00:00 America/New_York'
    after = sorted(i for i in rows if rows[i][0] > late)
    before = sorted(i for i in rows if rows[i][0] < early)
    assert after == [2, 3] and before == [7]   # the names s7_01.req.out prints
    out = {}
    # s7: T2 reads the late shows and updates the early ones, T3 the other
    # way round; T2 commits first, so T3's early-date range holds T2's keys
    out["s7"] = dict(
        txns={
            "T2": dict(reads=[rng_("shows", 1, K(late), None, rflag=1),
                              rng_("shows", 1, None, K(early), lflag=1)], writes=upd(before, 11000)),
            "T3": dict(reads=[rng_("shows", 1, None, K(early), lflag=1),
                              rng_("shows", 1, K(late), None, rflag=1)], writes=upd(after, 12000)),
        },
        events=[["begin", "T2"], ["begin", "T3"], ["commit", "T2"], ["commit", "T3"]],
        expect_fail=["T3"])
    hi_dec, lo_dec = 53210, 21200               # '5.321', '2.1200'
    big = sorted(i for i in rows if rows[i][1] > hi_dec)
    small = sorted(i for i in rows if rows[i][1] < lo_dec)
    assert big == [8, 12] and small == [1, 2, 7]   # s8_01.req.out's names
    # s8: the same skew over KEY_DEC; T1 commits first, T2's dec > 5.321
    # range holds the KEY_DEC keys T1 re-logged
    out["s8"] = dict(
        txns={
            "T1": dict(reads=[rng_("shows", 2, K(hi_dec), None, rflag=1),
                              rng_("shows", 2, None, K(lo_dec), lflag=1)], writes=upd(big, 13000)),
            "T2": dict(reads=[rng_("shows", 2, None, K(lo_dec), lflag=1),
                              rng_("shows", 2, K(hi_dec), None, rflag=1)], writes=upd(small, 14000)),
        },
        events=[["begin", "T1"], ["begin", "T2"], ["commit", "T1"], ["commit", "T2"]],
        expect_fail=["T2"])
    return out


def main():
    sc = scenarios()
    for name, s in sc.items():
        path = os.path.join(REF, f"{name}_01.req.out")
        n = sum(1 for line in open(path) if re.search(r"not serializable", line))
        s["reference_failures"] = n
        s["reference_file"] = f"tests/serialstep.test/{name}_01.req.out"
        assert n == len(s["expect_fail"]), (name, n, s["expect_fail"])
    with open(os.path.join(HERE, "serialstep.json"), "w") as f:
        json.dump(sc, f, indent=1, sort_keys=True)
    print("wrote", len(sc), "scenarios")


if __name__ == "__main__":
    main()
