#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the REFERENCE itself.

Run in the build container (needs /root/reference):

    make -C oracle all ref && python tests/golden/gen_golden.py

Expected outputs come from oracle/_ref/libref_mtcp_csum.so, i.e. the
reference's own compiled ``TCPCalcChecksum`` (mtcp/src/tcp_util.c:244-277)
and ``ip_fast_csum`` (io_engine/include/ps.h:66-95), driven in the RX order
of ip_in.c:21-59 / tcp_in.c:1208-1241 and the TX order of ip_out.c:143-173 /
tcp_out.c:244,323-333.  Inputs are seeded synthetic data.  Output files are
plain data (.npz without pickles, .json):

* kat.json        SURVEY.md §4 known answers, re-derived from the reference
* tcp_fn.npz      element-wise TCPCalcChecksum vectors (len 0..1600 + large)
* ip_fn.npz       element-wise ip_fast_csum vectors (ihl 0..15, carry edges)
* frames_rx.npz   packed frames -> RX verdicts (every verdict path)
* frames_tx.npz   packed frames (garbage checks) -> TX status + check values
* icmp_fn.npz     element-wise ICMPChecksum vectors (mtcp/src/icmp.c:18-42),
                  odd lengths with junk after the last byte
* rss.npz         GetRSSHash / GetRSSCPUCore (mtcp/src/rss.c:44-115) over
                  random and edge 4-tuples, 13 queue counts x both mappings
* frames_l4.npz   ICMP + TCP frames -> RX verdicts with the ICMP flag, TX
                  fill with the ICMP flag, RSS hash/core of ACCEPT frames

``python tests/golden/gen_golden.py [name ...]`` regenerates only the named
files (default: all).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle_lib import RefHarness  # noqa: E402
from mtcp_amd import synth  # noqa: E402

SEED = 0x6D746370


def ipaddr(s: str) -> int:
    """Dotted quad -> uint32 as stored in memory (network order) read LE."""
    b = bytes(int(x) for x in s.split("."))
    return int.from_bytes(b, "little")


def gen_kat(R: RefHarness) -> dict:
    out = {}
    hdr = bytes.fromhex("45000073000040004011b861c0a80001c0a800c7")
    buf = np.frombuffer(hdr + bytes(64), dtype=np.uint8).copy()
    out["ip_valid_header"] = {"hex": hdr.hex(), "ihl": 5, "expect": R.ip_fast_csum_at(buf, 0, 5)}
    z = bytearray(hdr)
    z[10:12] = b"\0\0"
    buf = np.frombuffer(bytes(z) + bytes(64), dtype=np.uint8).copy()
    out["ip_zeroed_check"] = {"hex": bytes(z).hex(), "ihl": 5, "expect": R.ip_fast_csum_at(buf, 0, 5)}
    buf = np.frombuffer(hdr + bytes(64), dtype=np.uint8).copy()
    out["ip_ihl4_quirk"] = {"hex": hdr.hex(), "ihl": 4, "expect": R.ip_fast_csum_at(buf, 0, 4)}
    zb = np.zeros(128, dtype=np.uint8)
    out["tcp_zero_len0"] = {"hex": "", "len": 0, "saddr": 0, "daddr": 0,
                            "expect": R.tcp_calc_checksum_at(zb, 0, 0, 0, 0)}
    out["tcp_zero_len20"] = {"hex": "00" * 20, "len": 20, "saddr": 0, "daddr": 0,
                             "expect": R.tcp_calc_checksum_at(zb, 0, 20, 0, 0)}
    rng = np.random.default_rng(SEED)
    seg = rng.integers(0, 256, 41, dtype=np.uint8)
    a = np.concatenate([seg, np.array([0x00], np.uint8), np.zeros(8, np.uint8)])
    b = np.concatenate([seg, np.array([0xEE], np.uint8), np.zeros(8, np.uint8)])
    sa, da = ipaddr("10.0.0.1"), ipaddr("10.0.0.2")
    ea = R.tcp_calc_checksum_at(a, 0, 41, sa, da)
    eb = R.tcp_calc_checksum_at(b, 0, 41, sa, da)
    assert ea == eb, "odd tail must ignore the byte after the segment"
    out["tcp_odd_tail"] = {"hex": bytes(seg).hex(), "len": 41, "saddr": sa, "daddr": da,
                           "expect": ea}
    # SURVEY.md §4 values, re-checked against the reference here
    assert out["ip_valid_header"]["expect"] == 0x0000
    assert out["ip_zeroed_check"]["expect"] == 0x61B8
    assert out["ip_ihl4_quirk"]["expect"] == 0x0045
    assert out["tcp_zero_len0"]["expect"] == 0xF9FF
    assert out["tcp_zero_len20"]["expect"] == 0xE5FF
    return out


def gen_tcp_fn(R: RefHarness):
    rng = np.random.default_rng(SEED + 1)
    lens = list(range(0, 1024)) + list(range(1024, 1601, 7)) + [4095, 4096, 9001, 16384, 65534, 65535]
    n = len(lens)
    lens = np.array(lens, dtype=np.uint32)
    starts = rng.integers(0, 8, size=n) * 2          # even, any value mod 16
    slots = (starts + lens + 2 + 15) // 16 * 16 + 16
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(slots[:-1], out=off[1:])
    buf = rng.integers(0, 256, size=int(off[-1] + slots[-1]) + 64, dtype=np.uint8)
    # a few all-0xFF payloads to push the 32-bit accumulator high
    for i in np.nonzero(lens >= 16384)[0][:3]:
        buf[int(off[i]) + int(starts[i]): int(off[i]) + int(starts[i]) + int(lens[i])] = 0xFF
    saddr = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    daddr = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    saddr[:4] = [0, 0xFFFFFFFF, 0, 0xFFFFFFFF]
    daddr[:4] = [0, 0xFFFFFFFF, 0xFFFFFFFF, 0]
    item_off = off + starts.astype(np.uint64)
    expect = np.array([R.tcp_calc_checksum_at(buf, int(item_off[i]), int(lens[i]),
                                              int(saddr[i]), int(daddr[i])) for i in range(n)],
                      dtype=np.uint16)
    return dict(buf=buf, off=item_off, len=lens.astype(np.uint16), saddr=saddr, daddr=daddr,
                expect=expect)


def gen_ip_fn(R: RefHarness):
    rng = np.random.default_rng(SEED + 2)
    n = 2048
    slot = 80
    buf = rng.integers(0, 256, size=n * slot + 64, dtype=np.uint8)
    ihl = (np.arange(n) % 16).astype(np.uint8)
    start = np.where(np.arange(n) % 3 == 0, 0, 2).astype(np.uint64)   # 0 or 2 mod 4
    off = np.arange(n, dtype=np.uint64) * slot + start
    for i in range(0, n, 7):          # all-ones headers: maximal ADC carry chains
        buf[int(off[i]): int(off[i]) + 60] = 0xFF
    for i in range(3, n, 11):         # all-zero headers
        buf[int(off[i]): int(off[i]) + 60] = 0
    for i in range(5, n, 13):         # words near 0xFFFFFFFF / 0x00000001
        w = rng.choice(np.array([0xFFFFFFFF, 0xFFFFFFFE, 1, 0, 0x0001FFFF], dtype=np.uint64), 15)
        b = np.frombuffer(w.astype("<u4").tobytes(), dtype=np.uint8)
        buf[int(off[i]): int(off[i]) + 60] = b
    expect = np.array([R.ip_fast_csum_at(buf, int(off[i]), int(ihl[i])) for i in range(n)],
                      dtype=np.uint16)
    return dict(buf=buf, off=off, ihl=ihl, expect=expect)


def _frame_set(R: RefHarness, rng: np.random.Generator):
    """A list of (bytes, frame_len) covering every RX/TX path."""
    frames = []

    def tcp_frame(payload, doff=8, ihl=5, pad=0, fill=True):
        L = 14 + 4 * ihl + 4 * doff + payload
        f = rng.integers(0, 256, size=L + pad + 4, dtype=np.uint8)
        f[12], f[13] = 0x08, 0x00
        f[14] = 0x40 | ihl
        tot = L - 14
        f[16], f[17] = tot >> 8, tot & 0xFF
        f[20], f[21], f[22], f[23] = 0x40, 0, 64, 6
        ts = 14 + 4 * ihl
        f[ts + 12] = (doff << 4)
        f[ts + 13] = 0x10
        if doff >= 8:
            f[ts + 20:ts + 24] = [1, 1, 8, 10]
        if fill:
            st, _ = R.tx_fill_at(f, 0, L + pad)
            assert st == 0
        return f, L + pad

    # all payload lengths 0..160, then sparse up to 1448; doff 5 and 8
    for p in list(range(0, 161)) + list(range(161, 1449, 37)) + [1448]:
        frames.append(tcp_frame(p, doff=8 if p % 2 else 5))
    # Ethernet padding: 60-byte minimum frames carrying short segments
    for p in range(0, 6):
        f, L = tcp_frame(p, doff=5, pad=0)
        g = np.concatenate([f[:L], rng.integers(0, 256, 60 - L + 4, dtype=np.uint8)]) if L < 60 else f
        frames.append((g, max(L, 60)))
    # IMIX
    for L in synth.imix_lengths(120, seed=SEED):
        frames.append(tcp_frame(int(L) - 54, doff=5 if L < 66 else 8))
    # IP options: ihl 6..15
    for ihl in range(6, 16):
        for p in (0, 1, 33, 200):
            frames.append(tcp_frame(p, doff=8, ihl=ihl))
    # odd doff values (data offsets 5..15)
    for doff in range(5, 16):
        frames.append(tcp_frame(17, doff=doff))
    base_valid = len(frames)
    # single-byte corruptions anywhere past the Ethernet header
    for k in range(240):
        f, L = frames[int(rng.integers(0, base_valid))]
        g = f.copy()
        pos = int(rng.integers(14, L))
        g[pos] ^= int(rng.integers(1, 256))
        frames.append((g, L))
    # crafted verdict paths ------------------------------------------------
    def refill_ip(g, ihl=5):
        g[24] = g[25] = 0
        c = R.ip_fast_csum_at(g, 14, ihl)
        g[24], g[25] = c & 0xFF, c >> 8

    f, L = tcp_frame(40)
    for et in (0x0806, 0x86DD, 0x0000, 0x0008):
        g = f.copy(); g[12], g[13] = et >> 8, et & 0xFF; frames.append((g, L))
    for ver in (0, 6, 15):                      # version != 4, valid IP checksum
        g = f.copy(); g[14] = (ver << 4) | 5; refill_ip(g); frames.append((g, L))
    for proto in (1, 17, 0, 255):               # not TCP, valid IP checksum
        g = f.copy(); g[23] = proto; refill_ip(g); frames.append((g, L))
    for tot in (0, 1, 19):                      # tot_len < 20
        g = f.copy(); g[16], g[17] = tot >> 8, tot & 0xFF; frames.append((g, L))
    for tot in (20, 39, 20 + 4 * 8 - 1):        # tot_len < (ihl+doff)*4, valid IP csum
        g = f.copy(); g[16], g[17] = tot >> 8, tot & 0xFF; refill_ip(g); frames.append((g, L))
    for tot in (L - 14 + 1, L - 14 + 100, 65535):   # tot_len beyond the frame
        g = f.copy(); g[16], g[17] = tot >> 8, tot & 0xFF; refill_ip(g); frames.append((g, L))
    for ihl in range(0, 5):                     # ihl <= 4 quirk
        g = f.copy(); g[14] = 0x40 | ihl; frames.append((g, L))
        g = f.copy(); g[14] = ihl; g[15] = 0; frames.append((g, L))   # hw14 == 0 -> NOT_V4 path
    g = f.copy(); g[14] = 0; g[15] = 0; frames.append((g, L))
    for short in (0, 5, 13, 14, 20, 33):        # frames shorter than the headers
        frames.append((f.copy(), short))
    g = f.copy(); g[14] = 0x4F; refill_ip(g, 15); frames.append((g, 14 + 60))   # doff past frame
    g = f.copy(); g[14] = 0x4F; frames.append((g, 40))                          # options past frame
    for doff in (0, 1, 4):                      # doff < 5 passes the TCP length test
        g = f.copy(); ts = 34; g[ts + 12] = doff << 4; frames.append((g, L))
        h, L2 = tcp_frame(12, doff=5); h[34 + 12] = doff << 4
        h[50] = h[51] = 0
        c = R.tcp_calc_checksum_at(h, 34, L2 - 34, int.from_bytes(bytes(h[26:30]), "little"),
                                   int.from_bytes(bytes(h[30:34]), "little"))
        h[50], h[51] = c & 0xFF, c >> 8
        frames.append((h, L2))
    # check fields crafted to land on 0x0000 / 0xFFFF edge values
    for k in range(40):
        frames.append(tcp_frame(int(rng.integers(0, 300)), doff=8))
    return frames


def _pack(frames):
    lens = np.array([L for _, L in frames], dtype=np.uint16)
    slots = (np.array([max(L, len(f)) for f, L in frames]) + 63) // 64 * 64 + 64
    off = np.zeros(len(frames), dtype=np.uint64)
    np.cumsum(slots[:-1], out=off[1:])
    buf = np.zeros(int(off[-1] + slots[-1]), dtype=np.uint8)
    for (f, L), o in zip(frames, off):
        buf[int(o): int(o) + len(f)] = f
    return buf, off, lens


def gen_frames_rx(R: RefHarness):
    rng = np.random.default_rng(SEED + 3)
    buf, off, lens = _pack(_frame_set(R, rng))
    expect = np.array([R.rx_verdict_at(buf, int(o), int(L)) for o, L in zip(off, lens)],
                      dtype=np.uint8)
    return dict(buf=buf, off=off, len=lens, expect=expect)


def gen_frames_tx(R: RefHarness):
    rng = np.random.default_rng(SEED + 4)
    frames = _frame_set(R, rng)
    # garbage in the check fields: the fill must not depend on them
    for f, L in frames:
        if len(f) >= 26:
            f[24], f[25] = rng.integers(0, 256, 2)
        ihl = f[14] & 15 if len(f) > 14 else 0
        ts = 14 + 4 * ihl
        if len(f) >= ts + 18:
            f[ts + 16], f[ts + 17] = rng.integers(0, 256, 2)
    buf, off, lens = _pack(frames)
    filled = buf.copy()
    status = np.zeros(len(off), dtype=np.uint8)
    csums = np.zeros(len(off), dtype=np.uint32)
    for i, (o, L) in enumerate(zip(off, lens)):
        status[i], csums[i] = R.tx_fill_at(filled, int(o), int(L))
    return dict(buf=buf, off=off, len=lens, status=status, csums=csums,
                filled_sha256=np.frombuffer(hashlib.sha256(filled.tobytes()).digest(),
                                            dtype=np.uint8))


def gen_icmp_fn(R: RefHarness):
    rng = np.random.default_rng(SEED + 5)
    lens = list(range(0, 600)) + list(range(600, 1481, 11)) + [1472, 1473, 1480, 4095, 65535]
    n = len(lens)
    lens = np.array(lens, dtype=np.uint32)
    starts = rng.integers(0, 8, size=n) * 2
    slots = (starts + lens + 2 + 15) // 16 * 16 + 16
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(slots[:-1], out=off[1:])
    buf = rng.integers(0, 256, size=int(off[-1] + slots[-1]) + 64, dtype=np.uint8)
    for i in np.nonzero(lens >= 4095)[0]:
        buf[int(off[i]) + int(starts[i]): int(off[i]) + int(starts[i]) + int(lens[i])] = 0xFF
    item_off = off + starts.astype(np.uint64)
    expect = np.array([R.icmp_checksum_at(buf, int(item_off[i]), int(lens[i])) for i in range(n)],
                      dtype=np.uint16)
    return dict(buf=buf, off=item_off, len=lens.astype(np.uint16), expect=expect)


RSS_NQ = np.array([1, 2, 3, 4, 5, 6, 7, 8, 12, 16, 32, 64, 100], dtype=np.int32)


def gen_rss(R: RefHarness):
    rng = np.random.default_rng(SEED + 6)
    n = 1024
    sip = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    dip = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    sp = rng.integers(0, 1 << 16, size=n).astype(np.uint16)
    dp = rng.integers(0, 1 << 16, size=n).astype(np.uint16)
    # edges: all-zero, all-ones, and each single input bit
    sip[0], dip[0], sp[0], dp[0] = 0, 0, 0, 0
    sip[1], dip[1], sp[1], dp[1] = 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFF, 0xFFFF
    for b in range(96):
        k = 2 + b
        sip[k] = dip[k] = sp[k] = dp[k] = 0
        if b < 32:
            sip[k] = 1 << (31 - b)
        elif b < 64:
            dip[k] = 1 << (63 - b)
        elif b < 80:
            sp[k] = 1 << (79 - b)
        else:
            dp[k] = 1 << (95 - b)
    h = np.array([R.rss_hash(int(sip[i]), int(dip[i]), int(sp[i]), int(dp[i])) for i in range(n)],
                 dtype=np.uint32)
    core = np.zeros((len(RSS_NQ), 2, n), dtype=np.int32)
    for a, nq in enumerate(RSS_NQ):
        for e in (0, 1):
            core[a, e] = [R.rss_core(int(sip[i]), int(dip[i]), int(sp[i]), int(dp[i]), int(nq), e)
                          for i in range(n)]
    return dict(sip=sip, dip=dip, sp=sp, dp=dp, hash=h, nq=RSS_NQ, core=core)


def _l4_frame_set(R: RefHarness, rng: np.random.Generator):
    frames = []

    def icmp_frame(payload, ihl=5, typ=8, fill=True):
        L = 14 + 4 * ihl + 8 + payload
        f = rng.integers(0, 256, size=L + 4, dtype=np.uint8)
        f[12], f[13] = 0x08, 0x00
        f[14] = 0x40 | ihl
        tot = L - 14
        f[16], f[17] = tot >> 8, tot & 0xFF
        f[20], f[21], f[22], f[23] = 0x40, 0, 64, 1
        ts = 14 + 4 * ihl
        f[ts], f[ts + 1] = typ, 0
        if fill:
            st, _ = R.tx_fill_f_at(f, 0, L, 0x2)
            assert st == 5, st
        return f, L

    def tcp_frame(payload, ihl=5, doff=8):
        L = 14 + 4 * ihl + 4 * doff + payload
        f = rng.integers(0, 256, size=L + 4, dtype=np.uint8)
        f[12], f[13] = 0x08, 0x00
        f[14] = 0x40 | ihl
        tot = L - 14
        f[16], f[17] = tot >> 8, tot & 0xFF
        f[20], f[21], f[22], f[23] = 0x40, 0, 64, 6
        ts = 14 + 4 * ihl
        f[ts + 12] = doff << 4
        st, _ = R.tx_fill_f_at(f, 0, L, 0)
        assert st == 0
        return f, L

    def refill_ip(g, ihl=5):
        g[24] = g[25] = 0
        c = R.ip_fast_csum_at(g, 14, ihl)
        g[24], g[25] = c & 0xFF, c >> 8

    for p in list(range(0, 130)) + list(range(130, 1473, 41)) + [1472]:
        frames.append(icmp_frame(p, typ=(8, 0, 3, 11)[p % 4]))
    for ihl in range(6, 16):
        for p in (0, 1, 7, 64, 301):
            frames.append(icmp_frame(p, ihl=ihl))
    for p in range(0, 260, 3):                           # TCP: RSS over ACCEPT frames
        frames.append(tcp_frame(p, ihl=5 + (p % 7 == 0) * (p % 11), doff=5 + (p % 4)))
    base_valid = len(frames)
    for k in range(160):                                 # single-byte corruptions
        f, L = frames[int(rng.integers(0, base_valid))]
        g = f.copy()
        pos = int(rng.integers(14, L))
        g[pos] ^= int(rng.integers(1, 256))
        frames.append((g, L))
    f, L = icmp_frame(40)
    for tot in (20, 23, 24, 27, 28, 29, 35):              # short ICMP messages, valid IP csum
        for ihl in (5, 6):
            g = f.copy(); g[14] = 0x40 | ihl
            g[16], g[17] = tot >> 8, tot & 0xFF
            refill_ip(g, ihl); frames.append((g, L))
    for tot in (L - 14 + 1, L - 14 + 64, 65535):          # ICMP message past the frame
        g = f.copy(); g[16], g[17] = tot >> 8, tot & 0xFF; refill_ip(g); frames.append((g, L))
    for short in (34, 35, 38, 41):                        # frames cut inside the ICMP header
        g = f.copy(); tot = short - 14
        g[16], g[17] = tot >> 8, tot & 0xFF; refill_ip(g); frames.append((g, short))
    for k in range(20):                                   # checksums landing on 0x0000/0xFFFF
        frames.append(icmp_frame(int(rng.integers(0, 200))))
    return frames


def gen_frames_l4(R: RefHarness):
    rng = np.random.default_rng(SEED + 7)
    frames = _l4_frame_set(R, rng)
    buf, off, lens = _pack(frames)
    rx = np.array([R.rx_verdict_f_at(buf, int(o), int(L), 0x2) for o, L in zip(off, lens)],
                  dtype=np.uint8)
    rx_noflag = np.array([R.rx_verdict_f_at(buf, int(o), int(L), 0) for o, L in zip(off, lens)],
                         dtype=np.uint8)
    # RSS of ACCEPT frames: (saddr, daddr, source, dest) in host order
    rss_hash = np.zeros(len(off), dtype=np.uint32)
    rss_core = np.full((2, len(off)), 0xFFFF, dtype=np.int32)
    for i, (o, L) in enumerate(zip(off, lens)):
        if rx[i] != 0:
            continue
        f = buf[int(o):]
        ts = 14 + 4 * (int(f[14]) & 15)
        sip = int.from_bytes(bytes(f[26:30]), "big")
        dip = int.from_bytes(bytes(f[30:34]), "big")
        sp = int.from_bytes(bytes(f[ts:ts + 2]), "big")
        dp = int.from_bytes(bytes(f[ts + 2:ts + 4]), "big")
        rss_hash[i] = R.rss_hash(sip, dip, sp, dp)
        rss_core[0, i] = R.rss_core(sip, dip, sp, dp, 16, 0)
        rss_core[1, i] = R.rss_core(sip, dip, sp, dp, 6, 1)
    # TX with the ICMP flag over garbage check fields
    tx = buf.copy()
    for o, L in zip(off, lens):
        o = int(o)
        if L >= 26:
            tx[o + 24], tx[o + 25] = rng.integers(0, 256, 2)
        ts = 14 + 4 * (int(tx[o + 14]) & 15) if L > 14 else 0
        if L >= ts + 4 and ts:
            tx[o + ts + 2], tx[o + ts + 3] = rng.integers(0, 256, 2)
    filled = tx.copy()
    status = np.zeros(len(off), dtype=np.uint8)
    csums = np.zeros(len(off), dtype=np.uint32)
    for i, (o, L) in enumerate(zip(off, lens)):
        status[i], csums[i] = R.tx_fill_f_at(filled, int(o), int(L), 0x2)
    return dict(buf=buf, off=off, len=lens, rx=rx, rx_noflag=rx_noflag, rss_hash=rss_hash,
                rss_core=rss_core, rss_nq=np.array([16, 6], dtype=np.int32),
                rss_endian=np.array([0, 1], dtype=np.int32), tx=tx, tx_status=status,
                tx_csums=csums,
                tx_filled_sha256=np.frombuffer(hashlib.sha256(filled.tobytes()).digest(),
                                               dtype=np.uint8))


GENERATORS = (("tcp_fn", gen_tcp_fn), ("ip_fn", gen_ip_fn), ("frames_rx", gen_frames_rx),
              ("frames_tx", gen_frames_tx), ("icmp_fn", gen_icmp_fn), ("rss", gen_rss),
              ("frames_l4", gen_frames_l4))


def main() -> None:
    if not RefHarness.available():
        sys.exit("oracle/_ref/libref_mtcp_csum.so missing: run `make -C oracle ref` "
                 "in a container that has /root/reference")
    R = RefHarness()
    only = set(sys.argv[1:])
    if not only or "kat" in only:
        with open(os.path.join(HERE, "kat.json"), "w") as fh:
            json.dump(gen_kat(R), fh, indent=1, sort_keys=True)
    for name, fn in GENERATORS:
        if only and name not in only:
            continue
        d = fn(R)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print(name, {k: (v.shape, str(v.dtype)) for k, v in d.items()})


if __name__ == "__main__":
    main()
