"""The egress seam with frames as vproxy holds them.

GpuCsumBatch.defer must describe a partially parsed frame by its IP header fields (totalLength,
IHL, payloadLength, extension headers), not by its buffer: the buffer of a 60-B frame holds the
Ethernet padding, and initPartial leaves IPv4 options unparsed (tests/egressvec.py).  The mirror
(vproxy_amd/vswitch.py: egress_descriptor, EgressBatch.defer_frame) is checked here against the
oracle's restatement of the reference parser on the CPU, and end to end on the GPU: deferred,
flushed with in-place writes, and byte-equal to the oracle's full recompute.  A descriptor the
kernel rejects goes back to the native path (GpuCsumBatch.flush restores the chunk's flags).
"""
import numpy as np
import pytest

import egressvec as E
from oracle import oracle as O


def _batch():
    fs = E.frames()
    arena, offs = E.layout(fs)
    flags = [E.want_flags(f["ver"], f["proto"], i) for i, f in enumerate(fs)]
    return fs, arena, offs, flags


def test_egress_descriptor_follows_the_ip_header():
    """egress_descriptor == the oracle parser's view for every frame (padding excluded, options
    and extension headers skipped, L3 after an 802.1Q tag)."""
    from vproxy_amd import vswitch as S
    fs, arena, offs, flags = _batch()
    want = E.oracle_descriptors(fs, offs, flags)
    for i, (f, o) in enumerate(zip(fs, offs)):
        d = S.egress_descriptor(arena[o:o + 64], o, flags[i])
        assert d is not None
        assert d.tobytes() == want[i].tobytes(), (f["kind"], d, want[i])


def test_buffer_length_descriptors_corrupt_these_frames(orc):
    """The round-2 derivation (buffer length, getHeaderSize) writes different bytes into the
    frames than Java's recompute on every padded, optioned or trailer-carrying frame with an L4
    sum to write: the vectors tell the two apart."""
    fs, arena, offs, flags = _batch()
    good = E.oracle_descriptors(fs, offs, flags)
    bad = E.buffer_length_descriptors(fs, offs, flags)
    a_good, a_bad = arena.copy(), arena.copy()
    orc.process(a_good, good, O.MODE_COMPUTE, write=True)
    orc.process(a_bad, bad, O.MODE_COMPUTE, write=True)
    differs = 0
    for i, o in enumerate(offs):
        if flags[i] & (O.F_L4 | O.F_L4P) and good[i].tobytes() != bad[i].tobytes():
            differs += not np.array_equal(a_good[o:o + 2048 - 384], a_bad[o:o + 2048 - 384])
    assert differs >= 0.9 * sum(1 for i in range(len(fs)) if flags[i] & (O.F_L4 | O.F_L4P)
                                and good[i].tobytes() != bad[i].tobytes())


@pytest.fixture(scope="module")
def V():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vproxy_amd import vpcsum
    vpcsum.lib()
    return vpcsum


@pytest.mark.gpu
@pytest.mark.parametrize("service", [False, True])
def test_egress_java_held_frames_on_gpu(V, orc, service):
    """Frames deferred the way GpuCsumBatch.defer now builds descriptors, flushed once (launched,
    or through the service grid from the registered umem), equal Java's full recompute byte for
    byte -- padding, options and extension-header bytes untouched."""
    from vproxy_amd import vswitch as S
    fs, arena, offs, flags = _batch()
    want = arena.copy()
    orc.process(want, E.oracle_descriptors(fs, offs, flags), O.MODE_COMPUTE, write=True)
    batch = S.EgressBatch(arena, capacity=len(fs), service_idle_us=20000 if service else 0)
    for o, fl in zip(offs, flags):
        assert batch.defer_frame(o, fl)
    assert batch.complete_tx() == len(fs)
    assert not batch.handed_back
    assert np.array_equal(arena, want)
    batch.close()


@pytest.mark.gpu
def test_egress_rejected_descriptor_is_handed_back(V, orc):
    """A frame the kernel refuses (a TCP segment too short to hold its checksum field) is not
    written and is handed back, the others are written; the flush reports only the GPU's frames."""
    from vproxy_amd import vswitch as S
    fs, arena, offs, flags = _batch()
    fs, offs, flags = fs[:40], offs[:40], flags[:40]
    arena = arena[:40 * E.CHUNK].copy()
    # frame 7 becomes IPv4/TCP with totalLength 30: 10 B of TCP, no room for the field at +16
    o = offs[7]
    hl = 18 if fs[7]["vlan"] else 14
    arena[o + hl] = 0x45
    arena[o + hl + 9] = 6
    arena[o + hl + 2:o + hl + 4] = [0, 30]
    flags[7] = O.F_IP | O.F_L4
    before7 = arena[o:o + 128].copy()
    good = [i for i in range(40) if i != 7]
    want = arena.copy()
    d_all = E.oracle_descriptors([fs[i] for i in good], [offs[i] for i in good], [flags[i] for i in good])
    orc.process(want, d_all, O.MODE_COMPUTE, write=True)
    batch = S.EgressBatch(arena, capacity=64)
    for oo, fl in zip(offs, flags):
        batch.defer_frame(oo, fl)
    assert batch.complete_tx() == 39
    assert batch.stats["rejected"] == 1
    # GpuCsumBatch.stats(): every deferred frame is accounted for, and the interface's csum_skip
    #  counts all 40, the GPU's and the handed-back one alike
    st = batch.stats
    assert (st["tx_csum_skip"], st["deferred"], st["gpu_handled"], st["bad_desc_handed_back"],
            st["small_flush_handed_back"]) == (40, 40, 39, 1, 0)
    assert len(batch.handed_back) == 1 and int(batch.handed_back[0][0]["l3_off"]) == o + hl
    assert np.array_equal(arena[o:o + 128], before7)
    assert np.array_equal(arena, want)
    batch.close()


@pytest.mark.gpu
@pytest.mark.parametrize("service", [False, True])
def test_egress_frames_parsed_on_gpu(V, orc, service):
    """vpcsum_ctx_egress_frames (FrameEgressBatch / VPCsum.egressFrames): only the frame offsets,
    the frame lengths as the TX ring sends them (padding and trailers included) and per-frame flags
    go to the GPU, which places L3 / L4 itself (a parse kernel and a checksum kernel, or the service
    grid's parse + sum per frame).  The umem equals the oracle's full recompute of the same frames,
    byte for byte."""
    from vproxy_amd import vswitch as S
    fs, arena, offs, flags = _batch()
    want = arena.copy()
    orc.process(want, E.oracle_descriptors(fs, offs, flags), O.MODE_COMPUTE, write=True)
    b = S.FrameEgressBatch(arena, capacity=len(fs), service_idle_us=20000 if service else 0)
    for f, o, fl in zip(fs, offs, flags):
        assert b.defer(o, len(f["frame"]), fl)
    assert b.complete_tx() == len(fs) and not b.handed_back
    assert np.array_equal(arena, want)
    assert b.ctx.stats()["service_batches"] == (1 if service else 0)
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("service", [False, True])
def test_egress_frames_refusals(V, orc, service):
    """Frames the GPU cannot honour are refused whole -- S_BAD_DESC, nothing written -- and handed
    back: an IPv4 header sum asked of IPv6, a pseudo-header sum asked of ICMPv4 (it has none), an
    ARP frame, a frame cut inside its IPv4 header, F_L4 and F_L4P together, F_RAW.  The others of
    the same flush are written."""
    from vproxy_amd import vswitch as S
    fs, arena, offs, flags = _batch()
    v6 = next(i for i, f in enumerate(fs) if f["ver"] == 6 and f["proto"] == 6)
    icmp4 = next(i for i, f in enumerate(fs) if f["ver"] == 4 and f["proto"] == 1)
    v4a, v4b, v4c, v4d = [i for i, f in enumerate(fs) if f["ver"] == 4 and f["proto"] == 6][:4]
    lens = [len(f["frame"]) for f in fs]
    bad = {v6: O.F_IP | O.F_L4, icmp4: O.F_L4P, v4a: O.F_L4 | O.F_L4P, v4b: O.F_RAW}
    for i, fl in bad.items():
        flags[i] = fl
    hl = 18 if fs[v4c]["vlan"] else 14
    arena[offs[v4c] + hl - 2:offs[v4c] + hl] = [0x08, 0x06]      # ARP
    bad[v4c] = flags[v4c]
    lens[v4d] = (18 if fs[v4d]["vlan"] else 14) + 12               # cut inside the IPv4 header
    bad[v4d] = flags[v4d]
    good = [i for i in range(len(fs)) if i not in bad]
    want = arena.copy()
    orc.process(want, E.oracle_descriptors([fs[i] for i in good], [offs[i] for i in good],
                                           [flags[i] for i in good]), O.MODE_COMPUTE, write=True)
    b = S.FrameEgressBatch(arena, capacity=len(fs), service_idle_us=20000 if service else 0)
    for o, L, fl in zip(offs, lens, flags):
        b.defer(o, L, fl)
    assert b.complete_tx() == len(good)
    assert sorted(x[0] for x in b.handed_back) == sorted(offs[i] for i in bad)
    assert np.array_equal(arena, want)
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("idle_us", [5000, 40])
def test_egress_frames_service_flushes(V, orc, idle_us):
    """Raw-frame flushes of 1..512 frames through the service grid (svc_frame_packet: each frame's
    first 384 B staged, parsed by lane 0, summed by the wave), consecutive batches over the 220
    vector frames (802.1Q, IPv4 options, IPv6 extension headers, padding, trailers) and a random
    stream, some frames refused (an ARP EtherType, flags a frame cannot honour): every status and
    every byte of the umem equals the launched path's (parse kernel + checksum kernel), itself
    pinned to the oracle above; the grid leaves between most flushes with idle_us = 40."""
    import time
    fs, arena, offs, flags = _batch()
    lens = np.array([len(f["frame"]) for f in fs], np.uint32)
    rng = np.random.default_rng(idle_us)
    fl = np.array(flags, np.uint8)
    fl[rng.random(len(fl)) < 0.05] = O.F_IP | O.F_L4P                 # refused where it cannot apply
    a_svc, a_ref = arena.copy(), arena.copy()
    c_svc = V.Context(0, max_arena=arena.nbytes, max_pkts=len(fs))
    c_ref = V.Context(0, max_arena=arena.nbytes, max_pkts=len(fs))
    c_svc.register(a_svc)
    c_ref.register(a_ref)
    c_svc.set_service(idle_us)
    offs = np.array(offs, np.uint64)
    iters = 40
    for it in range(iters):
        b = int(rng.choice([1, 2, 3, 4, 17, 64, 220]))
        idx = rng.choice(len(fs), b, replace=False) if b < len(fs) else np.arange(len(fs))
        o, L, f = offs[idx], lens[idx], fl[idx]
        out_s, st_s = c_svc.egress_frames(a_svc, o, L, f)
        out_r, st_r = c_ref.egress_frames(a_ref, o, L, f)
        assert np.array_equal(st_s, st_r), it
        assert np.array_equal(out_s, out_r), it
        assert np.array_equal(a_svc, a_ref), it
        t_end = time.perf_counter() + float(rng.integers(0, 3 * idle_us)) * 1e-6
        while time.perf_counter() < t_end:
            pass
    assert c_svc.stats()["service_batches"] == iters and c_ref.stats()["service_batches"] == 0
    c_svc.close()
    c_ref.close()


def test_egress_descriptor_random_frames():
    """2000 random frames as vproxy could hold them (IPv4 with IHL 5-15, IPv6 with 0 or 1 extension
    header, TCP / UDP / ICMP / ICMPv6 / other, 802.1Q or not, 0-40 B of padding or trailer): for
    every frame the reference's parser accepts, the mirror's descriptor equals the oracle's."""
    from vproxy_amd import vswitch as S
    rng = np.random.default_rng(2024)
    n_ok = 0
    for i in range(2000):
        vlan = bool(rng.integers(0, 2))
        ver = 4 if rng.random() < 0.6 else 6
        proto = int(rng.choice([6, 17, 1, 58, 47]))
        l4len = int(rng.integers(20, 300))
        if ver == 4:
            l3 = E._ipv4(rng, proto, l4len, int(rng.integers(5, 16)))
        else:
            l3 = E._ipv6(rng, proto, l4len, None if rng.random() < 0.5 else int(rng.integers(0, 64)))
        f = E._ether(rng, l3, ver, vlan, trailer=int(rng.integers(0, 41)))
        info, _ = O.parse_ether(f)
        if info is None:
            continue
        n_ok += 1
        fl = O.desc_flags_for(info)
        d = S.egress_descriptor(np.frombuffer(f[:64], np.uint8), 1000, fl)
        want = (1000 + info.l3_off, info.l3_len, info.l4_off, info.ver, info.proto, fl)
        got = (int(d["l3_off"]), int(d["l3_len"]), int(d["l4_off"]), int(d["l3_ver"]), int(d["l4_proto"]), int(d["flags"]))
        assert got == want, (i, got, want)
    assert n_ok > 1500


@pytest.mark.gpu
def test_egress_counters_small_flush_and_frames(V, orc):
    """The counters of both egress mirrors (GpuCsumBatch.stats in Java): a flush below the small-
    flush threshold hands its frames back and counts them as such; the raw-frame batch counts GPU
    frames and refusals; frames without dirty sums are not counted as skipped."""
    from vproxy_amd import vswitch as S
    fs, arena, offs, flags = _batch()
    b = S.EgressBatch(arena.copy(), capacity=16, small_flush=5)
    for o, fl in zip(offs[:3], flags[:3]):
        assert b.defer_frame(o, fl)
    assert not b.defer_frame(offs[3], 0)          # nothing dirty: the chunk keeps flags 0
    assert b.complete_tx() == 0
    st = b.stats
    assert (st["tx_pkts"], st["tx_csum_skip"], st["deferred"], st["gpu_handled"], st["small_flush_handed_back"],
            st["flushes"]) == (4, 3, 3, 0, 3, 0)
    b.close()
    a2 = arena.copy()
    fb = S.FrameEgressBatch(a2, capacity=64)
    for f, o, fl in zip(fs[:20], offs[:20], flags[:20]):
        assert fb.defer(o, len(f["frame"]), fl)
    fb.defer(offs[20], 10, flags[20])             # 10 B: no IP header, the GPU refuses it
    assert fb.complete_tx() == 20
    assert (fb.stats["tx_csum_skip"], fb.stats["deferred"], fb.stats["gpu_handled"],
            fb.stats["bad_desc_handed_back"], fb.stats["flushes"]) == (21, 21, 20, 1, 1)
    fb.close()


def test_egress_descriptor_short_frames_and_ext_chains():
    """egress_descriptor never reads past the bytes it is given (a frame within 64 B of the arena
    end), and an IPv6 chain of two extension headers yields the second header as l4_proto (refused
    by the kernel, so handed back), as the GPU parser refuses such a frame."""
    from vproxy_amd import vswitch as S
    assert S.egress_descriptor(np.zeros(10, np.uint8), 0, 3) is None
    v4 = np.zeros(30, np.uint8)
    v4[12:14] = [0x08, 0x00]
    assert S.egress_descriptor(v4, 0, 3) is None            # 16 B of a 20-B IPv4 header
    v6 = np.zeros(64, np.uint8)
    v6[12:14] = [0x86, 0xdd]
    v6[14] = 0x60
    v6[14 + 4:14 + 6] = [0, 24]
    v6[14 + 6] = 0                                        # hop-by-hop ...
    v6[14 + 40] = 60                                      # ... then destination options
    d = S.egress_descriptor(v6, 0, 2)
    assert int(d["l4_proto"]) == 60 and int(d["l4_off"]) == 48
    assert S.egress_descriptor(v6[:54], 0, 2) is None      # the extension header cut off


@pytest.mark.gpu
def test_egress_frames_large_mixed_batch(V, orc):
    """A flush large and mixed enough for the checksum kernel's sampled grid and its workgroup-sorted
    units, reached through vpcsum_ctx_egress_frames: 150,000 C3 frames in
    2-KB umem frames, registered (zero-copy), per-frame flags from the parse (the kernel's flags
    override), every third frame asking for the L4 sum only.  The umem equals the oracle's full
    recompute."""
    from vproxy_amd import vswitch as S
    n, stride = 150_000, 2048
    arena, d = orc.synth(n, stride, 14, O.SYNTH_C3, O.SEED, 31)
    frames = arena.reshape(n, stride)
    frames[:, 12], frames[:, 13] = 0x08, 0x00          # Ethernet type IPv4 before each L3 packet
    d = d.copy()
    d["flags"][::3] = O.F_L4
    want = arena.copy()
    orc.process(want, d, O.MODE_COMPUTE, write=True, threads=8)
    b = S.FrameEgressBatch(arena, capacity=n)
    for i in range(n):
        assert b.defer(i * stride, 14 + int(d["l3_len"][i]), int(d["flags"][i]))
    assert b.complete_tx() == n and not b.handed_back
    assert np.array_equal(arena, want)
    b.close()
