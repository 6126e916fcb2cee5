"""The CPU oracle (oracle/csum_ref.c) against the reference's golden vectors.

tests/golden/ was produced by tests/golden/gen_golden.py from the reference's
own compiled TCPCalcChecksum (mtcp/src/tcp_util.c:244-277) and ip_fast_csum
(io_engine/include/ps.h:66-95); these tests pin the oracle to it.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle_lib import Oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def O():
    return Oracle()


def load(name):
    with np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


def test_kat(O):
    kat = json.load(open(os.path.join(GOLD, "kat.json")))
    for name, k in kat.items():
        data = bytes.fromhex(k["hex"])
        if name.startswith("ip_"):
            got = O.ip_fast_csum(data, k["ihl"])
        else:
            got = O.tcp_calc_checksum(data, k["len"], k["saddr"], k["daddr"])
        assert got == k["expect"], name
    # SURVEY.md §4 known answers
    assert kat["ip_zeroed_check"]["expect"] == 0x61B8
    assert kat["tcp_zero_len0"]["expect"] == 0xF9FF
    assert kat["tcp_zero_len20"]["expect"] == 0xE5FF


def test_tcp_fn_golden(O):
    d = load("tcp_fn")
    got = O.tcp_checksum_batch(d["buf"], d["off"], d["len"], d["saddr"], d["daddr"])
    np.testing.assert_array_equal(got, d["expect"])


def test_ip_fn_golden(O):
    d = load("ip_fn")
    got = O.ip_checksum_batch(d["buf"], d["off"], d["ihl"])
    np.testing.assert_array_equal(got, d["expect"])


def test_frames_rx_golden(O):
    d = load("frames_rx")
    got = O.verify_batch(d["buf"].copy(), d["off"], d["len"])
    np.testing.assert_array_equal(got, d["expect"])


def test_frames_rx_zero_bad_check_side_effect(O):
    """tcp_in.c:1237: a TCP checksum failure zeroes tcph->check."""
    d = load("frames_rx")
    buf = d["buf"].copy()
    got = O.verify_batch(buf, d["off"], d["len"], flags=1)
    np.testing.assert_array_equal(got, d["expect"])
    changed = np.nonzero(buf != d["buf"])[0]
    bad = np.nonzero(d["expect"] == 7)[0]
    assert len(bad) > 0
    allowed = set()
    for i in bad:
        o = int(d["off"][i]); ihl = int(d["buf"][o + 14]) & 15
        allowed |= {o + 14 + 4 * ihl + 16, o + 14 + 4 * ihl + 17}
    assert set(changed.tolist()) <= allowed


def test_frames_tx_golden(O):
    d = load("frames_tx")
    buf = d["buf"].copy()
    st, cs = O.compute_batch(buf, d["off"], d["len"])
    np.testing.assert_array_equal(st, d["status"])
    np.testing.assert_array_equal(cs, d["csums"])
    assert hashlib.sha256(buf.tobytes()).digest() == d["filled_sha256"].tobytes()


def test_tx_then_rx_accepts(O):
    """Property: no TX_OK frame fails either checksum on RX (the verify fold
    over a filled frame is 0).  Frames with version != 4 or a doff longer
    than the segment are filled by TX but stopped earlier by RX."""
    d = load("frames_tx")
    buf = d["buf"].copy()
    st, _ = O.compute_batch(buf, d["off"], d["len"])
    v = O.verify_batch(buf, d["off"], d["len"])
    assert not np.isin(v[st == 0], [3, 7]).any()
    assert (v[st == 0] == 0).mean() > 0.95


# ---- ICMPChecksum and RSS --------------------------------

def test_icmp_fn_golden(O):
    """icmp.c:18-42, incl. odd lengths (the reference object zero-extends the
    uninitialised high byte of odd_byte) and junk after the last byte."""
    d = load("icmp_fn")
    got = O.icmp_checksum_batch(d["buf"], d["off"], d["len"])
    np.testing.assert_array_equal(got, d["expect"])
    assert (d["len"] % 2 == 1).sum() > 300


def test_rss_golden(O):
    """rss.c:44-115 with the reference's built-in key: hash and core mapping."""
    d = load("rss")
    n = len(d["sip"])
    got = np.array([O.rss_hash(int(d["sip"][i]), int(d["dip"][i]), int(d["sp"][i]),
                               int(d["dp"][i])) for i in range(n)], dtype=np.uint32)
    np.testing.assert_array_equal(got, d["hash"])
    for a, nq in enumerate(d["nq"]):
        for e in (0, 1):
            core = [O.rss_core(int(d["sip"][i]), int(d["dip"][i]), int(d["sp"][i]),
                               int(d["dp"][i]), int(nq), e) for i in range(0, n, 3)]
            np.testing.assert_array_equal(core, d["core"][a, e, ::3])


def test_rss_default_key_is_the_reference_key(O):
    key = bytes([5] * 40)
    assert O.rss_hash(0x0A000001, 0x0A000002, 1234, 80, key=key) == \
        O.rss_hash(0x0A000001, 0x0A000002, 1234, 80)


def test_frames_l4_golden(O):
    d = load("frames_l4")
    got = O.verify_batch(d["buf"].copy(), d["off"], d["len"], flags=0x2)
    np.testing.assert_array_equal(got, d["rx"])
    got = O.verify_batch(d["buf"].copy(), d["off"], d["len"], flags=0)
    np.testing.assert_array_equal(got, d["rx_noflag"])
    for k in range(2):
        vd, h, q = O.classify_batch(d["buf"].copy(), d["off"], d["len"], int(d["rss_nq"][k]),
                                    int(d["rss_endian"][k]), flags=0x2)
        np.testing.assert_array_equal(vd, d["rx"])
        acc = vd == 0
        np.testing.assert_array_equal(h[acc], d["rss_hash"][acc])
        np.testing.assert_array_equal(q[acc], d["rss_core"][k][acc])
        assert (q[~acc] == 0xFFFF).all() and (h[~acc] == 0).all()
    tx = d["tx"].copy()
    st, cs = O.compute_batch(tx, d["off"], d["len"], flags=0x2)
    np.testing.assert_array_equal(st, d["tx_status"])
    np.testing.assert_array_equal(cs, d["tx_csums"])
    assert hashlib.sha256(tx.tobytes()).digest() == bytes(d["tx_filled_sha256"])
    # every verdict / status the ICMP path defines is covered
    assert {10, 11, 0, 3, 8} <= set(d["rx"].tolist())
    assert {0, 5, 6} <= set(d["tx_status"].tolist())
