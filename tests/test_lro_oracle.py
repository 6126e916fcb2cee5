"""Software LRO in the oracle: the merge rules
(oracle/csum_ref.h ref_gro_batch) and, where oracle/_ref is built, that every
merged frame passes the reference's own RX checks (refx_rx_verdict) and
carries the members' payloads in order."""
import numpy as np
import pytest

from mtcp_amd import synth
from oracle_lib import Oracle, RefHarness


@pytest.fixture(scope="module")
def O():
    return Oracle()


def stream(n, seed, **kw):
    O = Oracle()
    buf, off, lens = synth.tcp_streams(n, seed=seed, **kw)
    O.compute_batch(buf, off, lens)
    vd = O.verify_batch(buf.copy(), off, lens)
    assert (vd == 0).all()
    return buf, off, lens, vd


def payload(buf, o, L):
    f = buf[int(o):int(o) + int(L)]
    tot = (int(f[16]) << 8) | int(f[17])
    hl = 34 + 4 * (int(f[46]) >> 4)
    return f[hl:14 + tot]


def check_runs(buf, off, lens, out, oo, ol, hd):
    """Every head's output = the members' payloads behind the head's headers."""
    n = len(off)
    heads = np.nonzero(hd == np.arange(n))[0]
    for h in heads:
        members = np.nonzero(hd == h)[0]
        assert (members == np.arange(h, h + len(members))).all()
        m = out[int(oo[h]):int(oo[h]) + int(ol[h])]
        if len(members) == 1:
            np.testing.assert_array_equal(m, buf[int(off[h]):int(off[h]) + int(lens[h])])
            continue
        pl = np.concatenate([payload(buf, off[k], lens[k]) for k in members])
        hl = 34 + 4 * (int(m[46]) >> 4)
        np.testing.assert_array_equal(m[hl:], pl)
        assert ((int(m[16]) << 8) | int(m[17])) == len(m) - 14
    return heads


def test_streams_merge_and_stay_valid(O):
    buf, off, lens, vd = stream(6000, 3)
    out, oo, ol, hd = O.gro_batch(buf, off, lens, vd, 64, 16384)
    heads = check_runs(buf, off, lens, out, oo, ol, hd)
    assert len(heads) < len(off) / 3
    assert (ol[heads] <= 16384).all() and (ol[hd != np.arange(len(off))] == 0).all()
    # merged frames verify with the oracle ...
    v = O.verify_batch(out.copy(), oo[heads], ol[heads])
    assert (v == 0).all()
    # ... and with the reference's own RX checks
    if RefHarness.available():
        R = RefHarness()
        assert all(R.rx_verdict_at(out, int(oo[h]), int(ol[h])) == 0 for h in heads)


@pytest.mark.parametrize("window,max_len", [(1, 16384), (2, 65535), (64, 3000), (256, 65535)])
def test_window_and_length_limits(O, window, max_len):
    buf, off, lens, vd = stream(3000, 4, n_flows=2, run_mean=40.0)
    out, oo, ol, hd = O.gro_batch(buf, off, lens, vd, window, max_len)
    check_runs(buf, off, lens, out, oo, ol, hd)
    assert (ol <= max(max_len, int(lens.max()))).all()
    assert (hd // window == np.arange(len(off)) // window).all()     # runs stay in windows
    if window == 1:
        assert (hd == np.arange(len(off))).all()


def test_merge_breakers(O):
    """Each perturbation ends a run exactly where the rules say."""
    buf, off, lens, vd = stream(400, 5, n_flows=1, run_mean=1e9, payload_max=500)
    base = O.gro_batch(buf, off, lens, vd, 256, 65535)[3]
    assert (base[:150] == 0).all()       # one flow, in order: one run (up to 65535 B)
    cases = {
        "seq gap": lambda f: f.__setitem__(41, f[41] ^ 1),
        "ack differs": lambda f: f.__setitem__(45, f[45] ^ 1),
        "window differs": lambda f: f.__setitem__(49, f[49] ^ 1),
        "option differs": lambda f: f.__setitem__(60, f[60] ^ 1),
        "ip id jump": lambda f: f.__setitem__(19, f[19] ^ 0x40),
        "ttl differs": lambda f: f.__setitem__(22, 63),
        "tos differs": lambda f: f.__setitem__(15, 4),
        "fin flag": lambda f: f.__setitem__(47, 0x11),
        "more-fragments": lambda f: f.__setitem__(20, 0x60),
    }
    k = 100
    for name, fn in cases.items():
        b = buf.copy()
        fn(b[int(off[k]):])
        O.compute_batch(b, off, lens)                      # checks stay valid
        v = O.verify_batch(b.copy(), off, lens)
        hd = O.gro_batch(b, off, lens, v, 256, 65535)[3]
        assert hd[k] == k, name                            # frame k starts a new run
        assert hd[k - 1] == 0, name
    # PSH on a frame ends the run after it
    b = buf.copy()
    b[int(off[k]) + 47] = 0x18
    O.compute_batch(b, off, lens)
    hd = O.gro_batch(b, off, lens, O.verify_batch(b.copy(), off, lens), 256, 65535)[3]
    assert hd[k] == 0 and hd[k + 1] == k + 1
    # a frame that failed the RX verify is never merged
    v = vd.copy()
    v[k] = 7
    hd = O.gro_batch(buf, off, lens, v, 256, 65535)[3]
    assert hd[k] == k and hd[k + 1] == k + 1
