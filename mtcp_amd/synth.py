"""Synthetic mTCP frames (numpy) for tests, golden fixtures and bench.py.

Frame geometry follows what mTCP emits:

* Ethernet 14 B (``mtcp.h:42``), IPv4 20 B with ``ihl=5``, ``ttl=64``, DF,
  ``check`` (``ip_out.c:143-153``);
* TCP 20 B + options: non-SYN data/ACK segments carry NOP,NOP,TS(10) = 12 B,
  so ``doff=8`` (``tcp_out.c:22-61, 117-124``);
* payload up to 1448 B (``tcp_out.c:565``).

The BASELINE.json configurations are:

* C1: 64 B frames, ``tot_len=50``, ``doff=5``, 10 B payload, stride 64;
* C2: 1500 B frames, ``tot_len=1486``, ``doff=8``, 1434 B payload, stride 1536;
* C3: IMIX 64/576/1500 at 7:4:1, offsets = prefix sum of ALIGN(L, 64)
  (``io_engine/lib/pslib.c:146``).

Everything here is host-side numpy; checksum *values* are never computed
here (the GPU compute kernel or, in tests, the oracle fills them).
"""
from __future__ import annotations

import numpy as np

DEFAULT_SEED = 0x6D746370  # "mtcp" 

ETH_LEN = 14
IP_LEN = 20
TCP_LEN = 20


def align(x, a):
    return (x + a - 1) // a * a


def stride_for(frame_len: int) -> int:
    """Slot stride for fixed-size frames: 64 B for small frames (two per
    128 B line), else 128 B multiples (1500 B -> 1536 B)."""
    return 64 if frame_len <= 64 else align(frame_len, 128)


def _write_headers(buf2d: np.ndarray, rng: np.random.Generator, frame_len: np.ndarray,
                   doff: np.ndarray, ihl: int = 5) -> None:
    """Write Ethernet/IPv4/TCP headers into rows of ``buf2d`` (n x >=64)
    in place.  ``frame_len``/``doff`` are per-row arrays.  Check fields are 0."""
    n = buf2d.shape[0]
    b = buf2d
    b[:, 12] = 0x08
    b[:, 13] = 0x00
    b[:, 14] = 0x40 | ihl
    b[:, 15] = 0
    tot = (frame_len - ETH_LEN).astype(np.uint32)
    b[:, 16] = (tot >> 8) & 0xFF
    b[:, 17] = tot & 0xFF
    # id: random (bytes 18-19 already random); frag_off = DF
    b[:, 20] = 0x40
    b[:, 21] = 0x00
    b[:, 22] = 64
    b[:, 23] = 6
    b[:, 24] = 0
    b[:, 25] = 0
    # saddr/daddr 26..33 random already
    ts = ETH_LEN + 4 * ihl
    # ports, seq, ack random; doff byte, flags = ACK
    b[:, ts + 12] = (doff.astype(np.uint8) << 4)
    b[:, ts + 13] = 0x10
    b[:, ts + 16] = 0
    b[:, ts + 17] = 0
    b[:, ts + 18] = 0
    b[:, ts + 19] = 0
    has_ts = doff >= 8
    if has_ts.any():
        rows = np.nonzero(has_ts)[0]
        b[rows, ts + 20] = 1      # NOP
        b[rows, ts + 21] = 1      # NOP
        b[rows, ts + 22] = 8      # TCPOPT_TIMESTAMP
        b[rows, ts + 23] = 10     # TCPOLEN_TIMESTAMP
    del n


def fixed_frames(n: int, frame_len: int, stride: int | None = None,
                 seed: int = DEFAULT_SEED) -> tuple[np.ndarray, int]:
    """``n`` frames of ``frame_len`` bytes at fixed ``stride`` (flat uint8
    array of n*stride bytes, padding bytes random).  doff=5 for frames that
    only fit a bare header (< 66 B), else 8 (NOP,NOP,TS)."""
    stride = stride or stride_for(frame_len)
    assert stride >= frame_len and stride % 16 == 0 and frame_len >= 54
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 256, size=n * stride, dtype=np.uint8)
    b2 = buf.reshape(n, stride)
    doff = np.full(n, 5 if frame_len < 66 else 8, dtype=np.uint32)
    _write_headers(b2, rng, np.full(n, frame_len, dtype=np.uint32), doff)
    return buf, stride


def imix_lengths(n: int, seed: int = DEFAULT_SEED) -> np.ndarray:
    """IMIX 64/576/1500 at 7:4:1 (BASELINE.json configs[3])."""
    rng = np.random.default_rng(seed ^ 0x494D4958)
    u = rng.integers(0, 12, size=n)
    return np.where(u < 7, 64, np.where(u < 11, 576, 1500)).astype(np.uint16)


def packed_offsets(lengths: np.ndarray, a: int = 64) -> tuple[np.ndarray, int]:
    """pslib-style packing: offset[i] = sum of ALIGN(len[j], a), j < i."""
    slots = (lengths.astype(np.uint64) + (a - 1)) // a * a
    off = np.zeros(len(lengths), dtype=np.uint64)
    if len(lengths) > 1:
        np.cumsum(slots[:-1], out=off[1:])
    total = int(off[-1] + slots[-1]) if len(lengths) else 0
    return off, total


def packed_frames(lengths: np.ndarray, seed: int = DEFAULT_SEED,
                  ) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Variable-length TCP frames packed at 64 B-aligned offsets.  Returns
    (buf, off[u64], len[u16]).  Every frame >= 54 B carries valid headers."""
    lengths = np.asarray(lengths, dtype=np.uint16)
    assert (lengths >= 54).all()
    off, total = packed_offsets(lengths)
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 256, size=total + 64, dtype=np.uint8)
    # header region of each frame as a gathered 2-D view, written back
    idx = off[:, None].astype(np.int64) + np.arange(64)[None, :]
    hdr = buf[idx]
    doff = np.where(lengths < 66, 5, 8).astype(np.uint32)
    _write_headers(hdr, rng, lengths.astype(np.uint32), doff)
    buf[idx] = hdr
    return buf, off, lengths


def corrupt(buf: np.ndarray, off: np.ndarray, lengths: np.ndarray, frac_log2: int = 10,
            seed: int = DEFAULT_SEED) -> np.ndarray:
    """Flip one random byte (never the Ethernet header) in a seeded
    1/2^frac_log2 of frames.  Returns the indices of corrupted frames."""
    rng = np.random.default_rng(seed ^ 0xBAD)
    n = len(off)
    pick = np.nonzero(rng.integers(0, 1 << frac_log2, size=n) == 0)[0]
    lengths = np.asarray(lengths)
    for i in pick:
        L = int(lengths[i] if lengths.ndim else lengths)
        pos = int(rng.integers(ETH_LEN, L))
        flip = int(rng.integers(1, 256))
        buf[int(off[i]) + pos] ^= flip
    return pick


def fixed_frames_device(n: int, frame_len: int, stride: int | None = None,
                        seed: int = DEFAULT_SEED, device: str = "cuda"):
    """Same frame template as ``fixed_frames`` but generated directly in HBM
    with torch (bench.py: 1.5-6 GB per GPU never touches the host).  Returns
    (uint8 tensor of n*stride bytes, stride).  Check fields are 0."""
    import torch

    stride = stride or stride_for(frame_len)
    assert stride >= frame_len and stride % 16 == 0 and frame_len >= 54
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=device, generator=g)
    b = buf.view(n, stride)
    tot = frame_len - ETH_LEN
    doff = 5 if frame_len < 66 else 8
    fixed = {12: 0x08, 13: 0x00, 14: 0x45, 15: 0, 16: tot >> 8, 17: tot & 0xFF, 20: 0x40,
             21: 0, 22: 64, 23: 6, 24: 0, 25: 0, 46: doff << 4, 47: 0x10, 50: 0, 51: 0,
             52: 0, 53: 0}
    if doff == 8:
        fixed.update({54: 1, 55: 1, 56: 8, 57: 10})
    cols = torch.tensor(sorted(fixed), device=device)
    vals = torch.tensor([fixed[k] for k in sorted(fixed)], dtype=torch.uint8, device=device)
    b[:, cols] = vals
    return buf, stride


def icmp_fixed_frames(n: int, frame_len: int, stride: int | None = None,
                      seed: int = DEFAULT_SEED) -> tuple[np.ndarray, int]:
    """``n`` ICMP echo-request frames of ``frame_len`` bytes (>= 42: Ethernet
    + IPv4 + the 8 B icmphdr, icmp.h) at a fixed stride, as ICMPOutput builds
    them through IPOutputStandalone (ip_out.c:72-101, icmp.c:44-77).  Check
    fields are 0."""
    stride = stride or stride_for(frame_len)
    assert stride >= frame_len and stride % 16 == 0 and frame_len >= 42
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 256, size=n * stride, dtype=np.uint8)
    b = buf.reshape(n, stride)
    b[:, 12], b[:, 13], b[:, 14], b[:, 15] = 0x08, 0x00, 0x45, 0
    tot = frame_len - ETH_LEN
    b[:, 16], b[:, 17] = (tot >> 8) & 0xFF, tot & 0xFF
    b[:, 20], b[:, 21], b[:, 22], b[:, 23] = 0x40, 0, 64, 1
    b[:, 24] = b[:, 25] = 0
    b[:, 34], b[:, 35] = 8, 0          # ICMP_ECHO, code 0
    b[:, 36] = b[:, 37] = 0            # icmp_checksum
    return buf, stride


def to_icmp(buf: np.ndarray, off: np.ndarray, lengths: np.ndarray, which: np.ndarray) -> None:
    """Turn the selected TCP frames (valid headers, any ihl) into ICMP echo
    requests in place: protocol 1, type 8 / code 0 at the L4 offset.  Frame
    and IP lengths are kept, so every frame >= 14 + 4*ihl + 8 stays valid."""
    for i in np.asarray(which):
        o = int(off[i])
        ihl = int(buf[o + 14]) & 15
        ts = o + ETH_LEN + 4 * ihl
        buf[o + 23] = 1
        buf[ts], buf[ts + 1] = 8, 0


def tcp_streams(n: int, n_flows: int = 8, run_mean: float = 6.0, payload_max: int = 1448,
                seed: int = DEFAULT_SEED) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """A received burst of ``n`` TCP data segments from ``n_flows`` flows, in
    bursts of consecutive in-order segments per flow (geometric run lengths of
    mean ``run_mean``), the way an LRO / GRO engine sees them.  Each flow has
    fixed addresses, ports, ack, window and timestamp option; sequence numbers
    and IP ids continue from segment to segment.  The last segment of a run
    sometimes carries PSH.  Packed like ``packed_frames``; check fields 0."""
    rng = np.random.default_rng(seed)
    flows = []
    for _ in range(n_flows):
        flows.append(dict(sip=rng.integers(0, 256, 4, dtype=np.uint8),
                          dip=rng.integers(0, 256, 4, dtype=np.uint8),
                          sp=int(rng.integers(1024, 65536)), dp=int(rng.integers(1, 1024)),
                          seq=int(rng.integers(0, 1 << 32)), ack=int(rng.integers(0, 1 << 32)),
                          win=int(rng.integers(1, 65536)), ipid=int(rng.integers(0, 65536)),
                          ts=rng.integers(0, 256, 8, dtype=np.uint8)))
    segs = []
    while len(segs) < n:
        fl = flows[int(rng.integers(0, n_flows))]
        run = min(int(rng.geometric(1.0 / run_mean)), n - len(segs))
        for k in range(run):
            pl = payload_max if rng.random() < 0.7 else int(rng.integers(1, payload_max + 1))
            psh = k == run - 1 and rng.random() < 0.3
            segs.append((fl, pl, psh, fl["seq"], fl["ipid"]))
            fl["seq"] = (fl["seq"] + pl) & 0xFFFFFFFF
            fl["ipid"] = (fl["ipid"] + 1) & 0xFFFF
    lens = np.array([14 + 20 + 32 + s[1] for s in segs], dtype=np.uint16)
    off, total = packed_offsets(lens)
    buf = rng.integers(0, 256, size=total + 64, dtype=np.uint8)
    for i, (fl, pl, psh, seq, ipid) in enumerate(segs):
        o = int(off[i])
        f = buf[o:o + int(lens[i])]
        f[12], f[13], f[14], f[15] = 0x08, 0x00, 0x45, 0
        tot = int(lens[i]) - 14
        f[16], f[17] = tot >> 8, tot & 0xFF
        f[18], f[19] = ipid >> 8, ipid & 0xFF
        f[20], f[21], f[22], f[23] = 0x40, 0, 64, 6
        f[24] = f[25] = 0
        f[26:30] = fl["sip"]
        f[30:34] = fl["dip"]
        f[34], f[35], f[36], f[37] = fl["sp"] >> 8, fl["sp"] & 0xFF, fl["dp"] >> 8, fl["dp"] & 0xFF
        f[38:42] = np.frombuffer(seq.to_bytes(4, "big"), dtype=np.uint8)
        f[42:46] = np.frombuffer(fl["ack"].to_bytes(4, "big"), dtype=np.uint8)
        f[46], f[47] = 8 << 4, 0x18 if psh else 0x10
        f[48], f[49] = fl["win"] >> 8, fl["win"] & 0xFF
        f[50] = f[51] = f[52] = f[53] = 0
        f[54], f[55], f[56], f[57] = 1, 1, 8, 10
        f[58:66] = fl["ts"]
    return buf, off, lens


def packed_frames_device(lengths: np.ndarray, seed: int = DEFAULT_SEED, device: str = "cuda"):
    """``packed_frames`` generated in HBM with torch (C3 IMIX at 4M frames):
    returns (uint8 buffer, off[int64 tensor], len[int16 tensor], total bytes).
    Headers as ``fixed_frames_device`` per length (doff 5 below 66 B, else 8);
    check fields 0."""
    import torch

    lengths = np.asarray(lengths, dtype=np.uint16)
    assert (lengths >= 54).all()
    off_np, total = packed_offsets(lengths)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    buf = torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device=device, generator=g)
    off = torch.from_numpy(off_np.astype(np.int64)).to(device)
    L = torch.from_numpy(lengths.astype(np.int64)).to(device)
    tot = L - ETH_LEN
    big = L >= 66
    cols = {12: 0x08, 13: 0x00, 14: 0x45, 15: 0, 20: 0x40, 21: 0, 22: 64, 23: 6, 24: 0, 25: 0,
            47: 0x10, 50: 0, 51: 0, 52: 0, 53: 0}
    for c, v in cols.items():
        buf[off + c] = v
    buf[off + 16] = (tot >> 8).to(torch.uint8)
    buf[off + 17] = (tot & 0xFF).to(torch.uint8)
    buf[off + 46] = torch.where(big, 8 << 4, 5 << 4).to(torch.uint8)
    ob = off[big]
    for c, v in ((54, 1), (55, 1), (56, 8), (57, 10)):
        buf[ob + c] = v
    return buf, off, torch.from_numpy(lengths.view(np.int16)).to(device), total


def tcp_streams_device(n: int, frame_len: int = 1500, flows: int = 16, run: int = 8,
                       device: str = "cuda"):
    """An LRO workload in HBM: ``n`` data segments of ``frame_len`` bytes (66 B
    of headers with NOP,NOP,TS) at stride ``stride_for(frame_len)``, from
    ``flows`` flows arriving in runs of ``run`` in-order segments each (frame
    i: flow (i // run) % flows).  Sequence numbers and IP ids continue per
    flow.  Returns (buffer, stride); check fields 0."""
    import torch

    stride = stride_for(frame_len)
    buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=device)
    b = buf.view(n, stride)
    i = torch.arange(n, device=device, dtype=torch.int64)
    fl = (i // run) % flows
    sgi = (i // (run * flows)) * run + i % run
    pl = frame_len - 66
    seq = (fl * 1000003 + sgi * pl) & 0xFFFFFFFF
    ipid = sgi & 0xFFFF
    tot = frame_len - ETH_LEN

    def put(col, val):
        b[:, col] = (val if torch.is_tensor(val) else torch.full_like(i, val)).to(torch.uint8)

    for c, v in {12: 8, 13: 0, 14: 0x45, 15: 0, 16: tot >> 8, 17: tot & 0xFF, 20: 0x40, 21: 0,
                 22: 64, 23: 6, 24: 0, 25: 0, 26: 10, 27: 0, 28: 0, 30: 10, 31: 0, 32: 1, 33: 1,
                 34: 0x80, 36: 0, 37: 80, 42: 1, 43: 2, 44: 3, 45: 4, 46: 8 << 4, 47: 0x10,
                 48: 0x10, 49: 0, 50: 0, 51: 0, 52: 0, 53: 0, 54: 1, 55: 1, 56: 8,
                 57: 10}.items():
        put(c, v)
    put(18, ipid >> 8)
    put(19, ipid & 0xFF)
    put(29, fl)
    put(35, fl)
    for k in range(4):
        put(38 + k, (seq >> (24 - 8 * k)) & 0xFF)
    for k in range(58, 66):
        put(k, fl + k)
    return buf, stride
