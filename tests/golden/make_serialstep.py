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
Index keys follow db/types.c:766-771 (0x08 + big-endian, sign bit flipped).
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
