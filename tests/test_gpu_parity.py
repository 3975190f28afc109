"""GPU parity: libvpcsum.so (HIP, gfx950) vs the CPU oracle, bit-exact, through the C-ABI.

Small cases compare every output word/status/byte with the oracle; the full-size C2 batch
(1M x 1500 B) is checked through size-independent properties (compute+write -> verify all OK,
idempotence) plus a random sample of packets against the oracle.
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from pcaputil import l3_offset, read_pcap

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def V():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vproxy_amd import vpcsum
    vpcsum.lib()
    return vpcsum


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().cuda()


def gpu_compute(V, arena_np, desc_np, mode=O.MODE_COMPUTE, team_log2=0, write=False):
    import torch
    arena = dev(arena_np.copy())
    d = V.desc_to_tensor(desc_np)
    n = len(desc_np)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.compute(arena, d, n, out, st, mode | (O.MODE_WRITE if write else 0), team_log2)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32), st.cpu().numpy(), arena.cpu().numpy()


def kat_batch():
    kats = json.load(open(os.path.join(GOLD, "kat.json")))["kats"]
    frames, infos = [], []
    for k in kats:
        fr = bytes.fromhex(k["hex"])
        info = O.parse_ether(fr)[0] if k["layer"] == "ether" else O.parse_l3(fr, 0, len(fr))[0]
        frames.append(fr)
        infos.append([info])
        if "inner_l3_off" in k:
            infos[-1].append(O.parse_l3(fr, k["inner_l3_off"], len(fr) - k["inner_l3_off"])[0])
    return kats, frames, infos


def pack(frames, infos, stride=None, pad=0):
    stride = stride or (max(len(f) for f in frames) + 64 + pad)
    arena = np.zeros(stride * len(frames), np.uint8)
    rows = []
    for i, (fr, inf) in enumerate(zip(frames, infos)):
        base = i * stride + pad
        arena[base:base + len(fr)] = np.frombuffer(fr, np.uint8)
        for x in inf:
            rows.append((base + x.l3_off, x.l3_len, x.l4_off, x.ver, x.proto, O.desc_flags_for(x), 0))
    desc = np.array(rows, dtype=O.DESC_DTYPE)
    return arena, desc


@pytest.mark.parametrize("pad", [0, 1, 2, 3, 14, 15, 398])
@pytest.mark.parametrize("team", [0, 2, 3, 5, 6, 9, 12, 40, 41, 43, 45, 46, 47, 48, 49, 50, 54, 58, 62, 66, 70, 74])
def test_kats_on_gpu(V, orc, pad, team):
    kats, frames, infos = kat_batch()
    arena, desc = pack(frames, infos, pad=pad)
    out, st, _ = gpu_compute(V, arena, desc, O.MODE_VERIFY, team)
    oout, ost = orc.process(arena, desc, O.MODE_VERIFY)
    assert np.array_equal(out, oout)
    assert np.array_equal(st, ost)
    # pinned values from TestPacket.java
    j = 0
    for k, inf in zip(kats, infos):
        pin = k["pinned"]
        if "ip" in pin:
            assert out[j] & 0xFFFF == pin["ip"]
        if "l4" in pin:
            assert out[j] >> 16 == pin["l4"]
        if "inner_ip" in pin:
            assert out[j + 1] & 0xFFFF == pin["inner_ip"] and out[j + 1] >> 16 == pin["inner_l4"]
        j += len(inf)
    assert np.all(st & O.S_DONE)


def test_pcap_verify_on_gpu(V, orc):
    frames, infos = [], []
    for fn in sorted(os.listdir(os.path.join(GOLD, "pcap"))):
        lt, pkts = read_pcap(os.path.join(GOLD, "pcap", fn))
        for p in pkts:
            off = l3_offset(lt, p)
            if off is None:
                continue
            info, err = O.parse_l3(p, off, len(p) - off)
            assert err is None
            frames.append(p)
            infos.append([info])
    arena, desc = pack(frames, infos)
    out, st, _ = gpu_compute(V, arena, desc, O.MODE_VERIFY)
    oout, ost = orc.process(arena, desc, O.MODE_VERIFY)
    assert np.array_equal(out, oout) and np.array_equal(st, ost)
    assert len(desc) == 31
    assert int(np.sum(st & O.S_IP_OK > 0)) == 31
    assert int(np.sum(st & O.S_L4_OK > 0)) == 19   # 12 CHECKSUM_PARTIAL host-TX frames fail


@pytest.mark.parametrize("workload", [O.SYNTH_C1, O.SYNTH_C2, O.SYNTH_C3, O.SYNTH_C4, O.SYNTH_FUZZ, O.SYNTH_C5])
@pytest.mark.parametrize("pad", [0, 1, 14, 398])
def test_synth_matches_oracle_and_checksums(V, orc, workload, pad):
    import torch
    n = 600 if workload in (O.SYNTH_C4, O.SYNTH_FUZZ) else 3000
    maxlen = 9000 if workload in (O.SYNTH_C4, O.SYNTH_FUZZ) else 1500
    stride = ((pad + maxlen + 63) // 64) * 64
    arena_o, desc_o = orc.synth(n, stride, pad, workload, O.SEED, first_index=12345)
    arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    V.synth(arena, n, stride, pad, workload, O.SEED, 12345, d)
    torch.cuda.synchronize()
    assert np.array_equal(arena.cpu().numpy(), arena_o), "GPU generator differs from oracle generator"
    assert np.array_equal(V.tensor_to_desc(d), desc_o)
    for team in (0, 2, 6, 9, 12, 40, 41, 43, 45, 46, 47, 48, 49, 50, 62, 66, 70, 74):
        out, st, written = gpu_compute(V, arena_o, desc_o, O.MODE_COMPUTE, team, write=True)
        a2 = arena_o.copy()
        oout, ost = orc.process(a2, desc_o, O.MODE_COMPUTE, write=True)
        assert np.array_equal(out, oout)
        assert np.array_equal(st, ost)
        assert np.array_equal(written, a2)
    # written frames verify clean
    out2, st2, _ = gpu_compute(V, written, desc_o, O.MODE_VERIFY)
    want = np.where(desc_o["flags"] & O.F_IP, O.S_IP_OK, 0) | O.S_L4_OK | O.S_DONE
    assert np.array_equal(st2 & ~np.uint8(O.S_UDP_NOCSUM), want.astype(np.uint8))
    assert np.array_equal(out2, out)


@pytest.mark.parametrize("team", [0, 8, 40, 45, 46, 47])
def test_raw_ranges(V, orc, team):
    rng = np.random.default_rng(5)
    lens = [0, 1, 2, 3, 5, 15, 16, 17, 31, 33, 63, 64, 65, 1499, 1500, 1501, 4097, 9000, 65535]
    arena = rng.integers(0, 256, 200000, dtype=np.uint8)
    arena[100000:110000] = 0
    arena[120000:130000] = 0xFF
    rows = []
    for L in lens:
        for off in (0, 1, 7, 100000 + 3, 120000 + 1, int(rng.integers(0, 100000))):
            if off + L <= len(arena):
                rows.append((off, L, 0, 0, 0, O.F_RAW, 0))
    desc = np.array(rows, dtype=O.DESC_DTYPE)
    out, st, _ = gpu_compute(V, arena, desc, team_log2=team)
    for r, o in zip(rows, out):
        assert o == O.csum(arena[r[0]:r[0] + r[1]].tobytes()), r


@pytest.mark.parametrize("team", [0, 40, 46, 47])
def test_bad_descriptors(V, orc, team):
    arena = np.zeros(4096, np.uint8)
    arena[0] = 0x45
    rows = [
        (4000, 200, 20, 4, 6, 3, 0),     # beyond arena
        (0, 19, 20, 4, 6, 3, 0),         # too short
        (0, 100, 22, 4, 6, 3, 0),        # l4_off not multiple of 4
        (0, 100, 20, 5, 6, 3, 0),        # bad version
        (0, 100, 20, 4, 58, 2, 0),       # ICMPv6 in IPv4
        (0, 100, 20, 6, 6, 1, 0),        # IP sum requested on IPv6
        (0, 30, 20, 4, 6, 2, 0),         # TCP segment shorter than its checksum field
        (2 ** 63, 100, 20, 4, 6, 3, 0),  # absurd offset
    ]
    desc = np.array(rows, dtype=O.DESC_DTYPE)
    out, st, after = gpu_compute(V, arena, desc, team_log2=team, write=True)
    oout, ost = orc.process(arena.copy(), desc)
    assert np.all(st == O.S_BAD_DESC) and np.all(ost == O.S_BAD_DESC)
    assert np.all(out == 0)
    assert np.array_equal(after, arena)


@pytest.mark.parametrize("team", [0, 8, 40, 41, 45, 46, 47, 48, 62, 66, 70, 74])
@pytest.mark.parametrize("mode", [O.MODE_COMPUTE, O.MODE_VERIFY])
def test_mixed_batch_bad_raw_interleaved(V, orc, team, mode):
    """Rejected, raw-range and slow-class (odd offset) descriptors interleaved with ordinary
    packets inside the same 64-packet groups: the size-sorted kernel must still hand every
    result back to its own descriptor."""
    n, stride, pad = 1000, 9088, 14
    arena, desc = orc.synth(n, stride, pad, O.SYNTH_FUZZ, O.SEED, 4242)
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)
    rng = np.random.default_rng(11)
    pick = rng.random(n)
    bad = pick < 0.1
    desc["l3_ver"][bad] = 5
    raw = (pick >= 0.1) & (pick < 0.2)
    desc["flags"][raw] = O.F_RAW
    odd = (pick >= 0.2) & (pick < 0.3)
    desc["l3_off"][odd] += 1                      # misaligned L3: slow class, garbage but defined
    desc["l3_len"][odd] = np.minimum(desc["l3_len"][odd], 8000)
    arena[rng.integers(0, arena.size, 500)] ^= 0x41   # some verify failures
    out, st, after = gpu_compute(V, arena, desc, mode, team, write=True)
    a2 = arena.copy()
    oout, ost = orc.process(a2, desc, mode, write=True)
    assert np.array_equal(st, ost)
    assert np.array_equal(out, oout)
    assert np.array_equal(after, a2)


def _nat_batch(orc, n, seed=3, corrupt=0.0, udp_zero=0.0, pad=0, workload=O.SYNTH_C3, packed=False):
    stride = 9088 if workload == O.SYNTH_FUZZ else 2048
    arena, desc = orc.synth(n, stride, pad, workload, O.SEED, 777)
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)       # valid input checksums
    rng = np.random.default_rng(seed)
    if packed:   # packets back to back (0-3 byte gaps): stores must never spill into a neighbour
        parts, offs, pos = [], [], pad
        parts.append(np.zeros(pad, np.uint8))
        for i in range(n):
            o, L = int(desc[i]["l3_off"]), int(desc[i]["l3_len"])
            offs.append(pos)
            parts.append(arena[o:o + L])
            gap = int(rng.integers(0, 4))
            parts.append(rng.integers(0, 256, gap, dtype=np.uint8))
            pos += L + gap
        arena = np.concatenate(parts)
        desc = desc.copy()
        desc["l3_off"] = offs
    if workload not in (O.SYNTH_C3, O.SYNTH_C5):
        udp_zero = 0.0
    rw = np.zeros(n, O.NAT4_DTYPE)
    rw["src"] = rng.integers(0, 256, (n, 4))
    rw["dst"] = rng.integers(0, 256, (n, 4))
    rw["sport"] = rng.integers(0, 256, (n, 2))
    rw["dport"] = rng.integers(0, 256, (n, 2))
    rw["mask"] = rng.integers(0, 64, n)
    rw["rsv"][:, 0] = rng.integers(0, 256, n)     # the VPCSUM_NAT_SET_TTL value
    for i in range(n):
        l3 = int(desc[i]["l3_off"])
        if rng.random() < corrupt:
            arena[l3 + 10] ^= 0x5A
            f = l3 + 20 + {6: 16, 17: 6, 1: 2}[int(desc[i]["l4_proto"])]
            arena[f + 1] ^= 0x33
        if desc[i]["l4_proto"] == 17 and rng.random() < udp_zero:
            arena[l3 + 26] = 0
            arena[l3 + 27] = 0
    return arena, desc, rw


@pytest.mark.parametrize("pad", [0, 1, 2, 14, 15])
@pytest.mark.parametrize("workload", [O.SYNTH_C1, O.SYNTH_C3, O.SYNTH_FUZZ, O.SYNTH_C5])
@pytest.mark.parametrize("packed", [False, True])
def test_nat_wide_and_scalar_kernels(V, orc, pad, workload, packed):
    """Both NAT kernels (wide LDS-staged and byte-access, nat_mode bit 8) against the Java
    restatement, at every window alignment, with packets packed back to back."""
    n = 1500 if workload == O.SYNTH_FUZZ else 3000
    arena, desc, rw = _nat_batch(orc, n, seed=pad + 17, udp_zero=0.1, pad=pad, workload=workload, packed=packed)
    want = arena.copy()
    want_st = orc.nat4_java(want, desc, rw)
    v4 = desc["l3_ver"] == 4
    assert np.all(want_st[~v4] == O.S_BAD_DESC)
    assert set(np.unique(want_st[v4])) <= {O.S_DONE, O.S_BAD_DESC | O.S_TTL_EXPIRED}
    # default, byte-access kernel (bit 8), wide kernel with 1 / 2 / 4 packets per lane (bits 12..14),
    # 4- and 6-chunk windows (bits 16..17: packets that do not fit 4 take the byte path), grids of
    # 3 and 16 workgroups per CU (bits 18..22); the lane layout (k_natw, bit 23) next to the default
    # quads (k_natq), and quads under a waves-per-EU bound of 6 / 8 (bits 24..25)
    for force_scalar in (0, 0x100, 0x1000, 0x2000, 0x3000, 0x10000, 0x20000, 0x23000, 0x20000 | (3 << 18),
                         0x20000 | (16 << 18), 0x800000, 0x801000, 0x823000, 0x1021000, 0x2002000):
        got, st = _gpu_nat(V, arena, desc, rw, V.NAT_RFC1624 | force_scalar)
        assert np.array_equal(st, want_st), force_scalar
        assert np.array_equal(got, want), force_scalar
        got, st = _gpu_nat(V, arena, desc, rw, V.NAT_STRICT_JAVA | force_scalar)
        assert np.array_equal(got, want), force_scalar
        assert np.array_equal(st & (O.S_BAD_DESC | O.S_TTL_EXPIRED), want_st & (O.S_BAD_DESC | O.S_TTL_EXPIRED))


def _gpu_nat(V, arena_np, desc, rw, mode):
    import torch
    arena = dev(arena_np.copy())
    st = torch.zeros(len(desc), dtype=torch.uint8, device="cuda")
    V.nat4(arena, V.desc_to_tensor(desc), dev(rw.view(np.uint8)), len(desc), st, mode)
    torch.cuda.synchronize()
    return arena.cpu().numpy(), st.cpu().numpy()


def _gpu_nat_rec(V, arena_np, desc, rw, mode):
    import torch
    arena = dev(arena_np.copy())
    rec = np.zeros(len(desc), V.NAT4R_DTYPE)
    rec["desc"], rec["rw"] = desc, rw
    st = torch.zeros(len(desc), dtype=torch.uint8, device="cuda")
    V.nat4r(arena, dev(rec.view(np.uint8)), len(desc), st, mode)
    torch.cuda.synchronize()
    return arena.cpu().numpy(), st.cpu().numpy()


@pytest.mark.parametrize("pad", [0, 2, 14])
@pytest.mark.parametrize("workload", [O.SYNTH_C3, O.SYNTH_FUZZ, O.SYNTH_C5])
@pytest.mark.parametrize("packed", [False, True])
def test_nat_records_against_java(V, orc, pad, workload, packed):
    """vpcsum_nat4r_async (vpcsum_nat4_rec_t: descriptor + IPv4 entry in one 32-B record) on every
    kernel shape equals the Java restatement byte for byte (IPv6 refused, TTL-expired refused,
    UDP stored 0 recomputed); the strict-Java mode is refused for records."""
    n = 1500 if workload == O.SYNTH_FUZZ else 3000
    arena, desc, rw = _nat_batch(orc, n, seed=pad + 71, udp_zero=0.1, pad=pad, workload=workload, packed=packed)
    want = arena.copy()
    want_st = orc.nat4_java(want, desc, rw)
    for tune in (0, 0x100, 0x1000, 0x3000, 0x20000, 0x23000, 0x800000, 0x801000, 0x20000 | (3 << 18)):
        got, st = _gpu_nat_rec(V, arena, desc, rw, V.NAT_RFC1624 | tune)
        assert np.array_equal(st, want_st), tune
        assert np.array_equal(got, want), tune
    with pytest.raises(V.VpcsumError, match="RFC1624"):
        _gpu_nat_rec(V, arena, desc, rw, V.NAT_STRICT_JAVA)


def test_nat_rfc1624_bit_exact_on_valid_input(V, orc):
    arena, desc, rw = _nat_batch(orc, 4000, udp_zero=0.1)
    want = arena.copy()
    want_st = orc.nat4_java(want, desc, rw)
    got, st = _gpu_nat(V, arena, desc, rw, V.NAT_RFC1624)
    assert np.array_equal(st, want_st)
    assert np.array_equal(got, want)


def test_nat_strict_java_on_invalid_input(V, orc):
    arena, desc, rw = _nat_batch(orc, 3000, seed=9, corrupt=0.3, udp_zero=0.2)
    want = arena.copy()
    orc.nat4_java(want, desc, rw)
    got, st = _gpu_nat(V, arena, desc, rw, V.NAT_STRICT_JAVA)
    assert np.array_equal(got, want)
    # RFC 1624 diverges exactly where the input was wrong -- documented behaviour
    got_fast, _ = _gpu_nat(V, arena, desc, rw, V.NAT_RFC1624)
    assert not np.array_equal(got_fast, want)


def _gpu_nat48(V, arena_np, desc, rw, mode):
    import torch
    arena = dev(arena_np.copy())
    st = torch.zeros(len(desc), dtype=torch.uint8, device="cuda")
    V.nat(arena, V.desc_to_tensor(desc), dev(rw.view(np.uint8)), len(desc), st, mode)
    torch.cuda.synchronize()
    return arena.cpu().numpy(), st.cpu().numpy()


def _nat4_of(rw48):
    """The 16-B IPv4 entries of 48-B ones (rsv[0] = the SET_TTL value)."""
    r4 = np.zeros(len(rw48), O.NAT4_DTYPE)
    r4["src"] = rw48["src"][:, :4]
    r4["dst"] = rw48["dst"][:, :4]
    r4["sport"] = rw48["sport"]
    r4["dport"] = rw48["dport"]
    r4["mask"] = rw48["mask"]
    r4["rsv"][:, 0] = rw48["ttl"]
    return r4


def test_nat_golden(V):
    """The reference's own checkPartialAndModify rewrites (setSrc / setDst 1.2.3.4 and ::2,
    setTtl(5), setHopLimit(5), setSrcPort / setDstPort(121)) and IPInputRoute's TTL decrement on
    the TestPacket frames: both entry formats, both kernels, RFC 1624 and strict Java."""
    d = json.load(open(os.path.join(GOLD, "nat.json")))
    assert {c["ver"] for c in d["cases"]} == {4, 6}
    for c in d["cases"]:
        fr = bytes.fromhex(c["before"])
        info, _ = O.parse_l3(fr, c["l3_off"], len(fr) - c["l3_off"])
        desc = np.array([(info.l3_off, info.l3_len, info.l4_off, info.ver, info.proto, O.desc_flags_for(info), 0)],
                        dtype=O.DESC_DTYPE)
        rw = np.frombuffer(bytes.fromhex(c["entry"]), O.NAT_DTYPE).copy()
        a = np.frombuffer(fr, np.uint8)
        for mode in (V.NAT_RFC1624, V.NAT_STRICT_JAVA, V.NAT_RFC1624 | 0x100, V.NAT_STRICT_JAVA | 0x100):
            got, st = _gpu_nat48(V, a, desc, rw, mode)
            assert got.tobytes().hex() == c["after"], (c["kat"], c["rewrite"], mode)
            assert st[0] == O.S_DONE
            got, st = _gpu_nat(V, a, desc, _nat4_of(rw), mode)
            if info.ver == 4:
                assert got.tobytes().hex() == c["after"], (c["kat"], c["rewrite"], mode, "nat4")
            else:   # the 16-B entry carries IPv4 addresses only: IPv6 is refused, untouched
                assert st[0] == O.S_BAD_DESC and got.tobytes() == fr


def _nat48_batch(orc, rng, n, pad=0, corrupt=0.0):
    """FUZZ packets (IPv4 with options, IPv6, TCP / UDP / ICMP / ICMPv6) with valid sums, 10% UDP
    stored 0, and random 48-B rewrites with every mask bit."""
    arena, desc = orc.synth(n, 9088, pad, O.SYNTH_FUZZ, O.SEED, int(rng.integers(0, 1 << 30)))
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)
    for d in desc:
        o, l4 = int(d["l3_off"]), int(d["l4_off"])
        if d["l4_proto"] == 17 and rng.random() < 0.1:
            arena[o + l4 + 6:o + l4 + 8] = 0
        if rng.random() < corrupt:
            arena[o + l4 + 1 + (int(d["l3_len"]) - l4) // 2] ^= 0x5A   # invalid L4 sums
    rw = np.zeros(n, O.NAT_DTYPE)
    rw.view(np.uint8).reshape(n, 48)[:, :38] = rng.integers(0, 256, (n, 38), dtype=np.uint8)
    rw["mask"] = rng.integers(0, 64, n)
    return arena, desc, rw


@pytest.mark.parametrize("pad", [0, 1, 2, 14])
def test_nat_v4_v6_against_java(V, orc, pad):
    """vpcsum_nat_async on IPv4 and IPv6: RFC 1624 equals Java's full recompute on valid input,
    strict Java equals it on any input; the wide kernel and the byte-access kernel agree."""
    rng = np.random.default_rng(100 + pad)
    arena, desc, rw = _nat48_batch(orc, rng, 1500, pad)
    want = arena.copy()
    want_st = orc.nat_java(want, desc, rw)
    for mode in (V.NAT_RFC1624, V.NAT_STRICT_JAVA, V.NAT_RFC1624 | 0x100, V.NAT_STRICT_JAVA | 0x100,
                 V.NAT_RFC1624 | 0x1000, V.NAT_RFC1624 | 0x3000):
        got, st = _gpu_nat48(V, arena, desc, rw, mode)
        assert np.array_equal(st, want_st), hex(mode)
        assert np.array_equal(got, want), hex(mode)
    # corrupted inputs: strict Java still matches, RFC 1624 diverges exactly there
    arena, desc, rw = _nat48_batch(orc, rng, 800, pad, corrupt=0.3)
    want = arena.copy()
    orc.nat_java(want, desc, rw)
    got, _ = _gpu_nat48(V, arena, desc, rw, V.NAT_STRICT_JAVA)
    assert np.array_equal(got, want)
    got, _ = _gpu_nat48(V, arena, desc, rw, V.NAT_RFC1624)
    assert not np.array_equal(got, want)


def test_nat_edge_packets_v6(V, orc):
    """The crafted edge packets (IPv6 extension headers with odd l4_off, ICMPv4 in IPv6, sums of
    0, UDP stored 0) under 48-B rewrites: wide window where it fits, byte access beyond it."""
    import edgevec as E
    pk = [p for p in E.edge_packets(np.random.default_rng(7)) if p["l3_len"] <= 9000]
    for pad in (0, 3):
        arena, desc = E.pack(pk, pad)
        rng = np.random.default_rng(pad)
        rw = np.zeros(len(desc), O.NAT_DTYPE)
        rw.view(np.uint8).reshape(-1, 48)[:, :38] = rng.integers(0, 256, (len(desc), 38), dtype=np.uint8)
        rw["mask"] = rng.integers(1, 64, len(desc))
        want = arena.copy()
        orc.nat_java(want, desc, rw)
        for mode in (V.NAT_RFC1624, V.NAT_STRICT_JAVA):
            got, st = _gpu_nat48(V, arena, desc, rw, mode)
            assert np.array_equal(got, want), (pad, mode)


@pytest.mark.parametrize("registered", [False, True])
def test_ctx_nat_submit(V, orc, registered):
    """vpcsum_ctx_nat_submit on host frames: staged (pageable arena: headers copied back at wait)
    and zero-copy (registered arena: rewritten in place), both modes, rejected descriptors
    untouched."""
    rng = np.random.default_rng(5 + registered)
    arena, desc, rw = _nat48_batch(orc, rng, 700, 14)
    desc = desc.copy()
    desc["l3_ver"][::50] = 5                 # rejected
    arena = np.concatenate([arena, np.zeros(4096, np.uint8)])
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=len(desc))
    if registered:
        ctx.register(arena)
    base = arena.copy()
    for mode in (V.NAT_RFC1624, V.NAT_STRICT_JAVA):
        a = arena if registered else base.copy()
        a[:] = base
        want = base.copy()
        wst = orc.nat_java(want, desc, rw)
        st = ctx.nat(a, desc, rw, mode)
        assert np.array_equal(st, wst), mode
        assert np.array_equal(a, want), mode
    ctx.close()


def test_parse_ether_matches_reference_rules(V):
    import torch
    frames = []
    for fn in sorted(os.listdir(os.path.join(GOLD, "pcap"))):
        lt, pkts = read_pcap(os.path.join(GOLD, "pcap", fn))
        if lt == 1:
            frames += pkts
    kats = json.load(open(os.path.join(GOLD, "kat.json")))["kats"]
    frames += [bytes.fromhex(k["hex"]) for k in kats if k["layer"] == "ether"]
    # VLAN-tagged, IPv6 with one ext header, truncated, non-IP, padded frames
    base = bytes.fromhex(kats[2]["hex"])
    frames.append(base[:12] + b"\x81\x00\x00\x05" + base[12:])
    frames.append(base + b"\x00" * 6)                        # Ethernet padding
    frames.append(base[:30])                                 # truncated
    frames.append(base[:12] + b"\x08\x06" + base[14:])       # ARP type
    v6 = bytes.fromhex(kats[1]["hex"])
    ext = bytes([58, 6]) + bytes(12)                         # hop-by-hop, hdrExtLen 6 -> 14 B
    v6x = bytearray(v6[:40] + ext + v6[40:])
    v6x[6] = 0
    pl = len(v6x) - 40
    v6x[4:6] = pl.to_bytes(2, "big")
    frames.append(bytes(12) + b"\x86\xdd" + bytes(v6x))
    frames.append(bytes(12) + b"\x86\xdd" + v6)
    offs, lens = [], []
    arena = bytearray()
    for f in frames:
        offs.append(len(arena))
        lens.append(len(f))
        arena += f + bytes((-len(f)) % 64)
    n = len(frames)
    a = dev(np.frombuffer(bytes(arena), np.uint8))
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.parse_ether(a, dev(np.array(offs, np.uint64)), dev(np.array(lens, np.uint32)), n, d, st)
    torch.cuda.synchronize()
    got = V.tensor_to_desc(d)
    stn = st.cpu().numpy()
    for i, f in enumerate(frames):
        info, err = O.parse_ether(f)
        if info is None:
            assert stn[i] == O.S_BAD_DESC, (i, err)
            continue
        assert stn[i] == 0
        g = got[i]
        assert int(g["l3_off"]) == offs[i] + info.l3_off
        assert (g["l3_len"], g["l4_off"], g["l3_ver"], g["l4_proto"]) == (info.l3_len, info.l4_off, info.ver, info.proto)
        assert g["flags"] == O.desc_flags_for(info)


def test_context_host_api(V, orc):
    arena, desc = orc.synth(5000, 2048, 14, O.SYNTH_C3, O.SEED, 99)
    want_out, want_st = orc.process(arena, desc, O.MODE_COMPUTE)
    ctx = V.Context(0, max_arena=16 << 20, max_pkts=8192)
    out, st = ctx.run(arena, desc)
    assert np.array_equal(out, want_out) and np.array_equal(st, want_st)
    # registered (page-locked) arena, in-place write, then verify through the same context
    ctx.register(arena)
    a2 = arena.copy()
    orc.process(a2, desc, O.MODE_COMPUTE, write=True)
    out = np.zeros(len(desc), np.uint32)
    t = ctx.submit(arena, desc, out, None, O.MODE_WRITE)
    ctx.wait(t)
    assert np.array_equal(arena, a2)
    out, st = ctx.run(arena, desc, O.MODE_VERIFY)
    assert np.all(st & O.S_L4_OK)
    ctx.unregister(arena)
    # two batches in flight
    ta = ctx.submit(arena, desc[:2000], oa := np.zeros(2000, np.uint32))
    tb = ctx.submit(arena, desc[2000:], ob := np.zeros(3000, np.uint32))
    ctx.wait(tb)
    ctx.wait(ta)
    assert np.array_equal(np.concatenate([oa, ob]), want_out)
    ctx.close()


def test_context_pipeline(V, orc):
    n, stride = 20000, 2048
    arena, desc = orc.synth(n, stride, 0, O.SYNTH_C2, O.SEED, 5)
    want, _ = orc.process(arena, desc)
    out = np.zeros(n, np.uint32)
    ctx = V.Context(0, max_arena=8 << 20, max_pkts=4096)
    ctx.register(arena)
    ctx.register(desc)
    ctx.register(out)
    ctx.pipeline(arena, stride, 1504, desc, out, chunks=8)
    assert np.array_equal(out, want)
    # MODE_WRITE: the checksum fields land in the host frames too
    want_arena = arena.copy()
    orc.process(want_arena, desc, O.MODE_COMPUTE, write=True)
    out[:] = 0
    ctx.pipeline(arena, stride, 1504, desc, out, mode=O.MODE_WRITE, chunks=8)
    assert np.array_equal(out, want) and np.array_equal(arena, want_arena)
    # a descriptor outside the copied part of its chunk's frames is refused, not read
    d2 = desc.copy()
    ctx.register(d2)   # registered until close: keep the array alive
    for i, bad in ((3000, 0), (7, 1600), (19999, n * stride)):
        d2[:] = desc
        d2["l3_off"][i] = bad
        with pytest.raises(V.VpcsumError, match="outside the copied frames"):
            ctx.pipeline(arena, stride, 1504, d2, out, chunks=8)
    ctx.close()
    del d2


def test_full_size_c2_properties(V, orc):
    """BASELINE config C2 at full size: 1,048,576 x 1500 B, stride 2048."""
    import torch
    n, stride = 1 << 20, 2048
    arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    V.synth(arena, n, stride, 0, O.SYNTH_C2, O.SEED, 0, d)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.compute(arena, d, n, out, st, O.MODE_WRITE)
    out2 = torch.zeros_like(out)
    V.compute(arena, d, n, out2, st, O.MODE_VERIFY)
    torch.cuda.synchronize()
    stn = st.cpu().numpy()
    assert np.all(stn == (O.S_DONE | O.S_IP_OK | O.S_L4_OK))
    assert torch.equal(out, out2)
    # random sample against the oracle (regenerated on the CPU from the same counters)
    rng = np.random.default_rng(11)
    idx = np.sort(rng.choice(n, 3000, replace=False))
    o = out.cpu().numpy().view(np.uint32)
    for i in idx[:3000]:
        a1, d1 = orc.synth(1, stride, 0, O.SYNTH_C2, O.SEED, int(i))
        w, _ = orc.process(a1, d1)
        assert o[i] == w[0]


@pytest.mark.parametrize("cfg", ["c1", "c2", "c3", "c4"])
def test_full_size_configs_equal_oracle(V, orc, cfg):
    """Every BASELINE checksum config at its full size (C1 1,048,576 x 64-B frames, C2 1,048,576 x
    1500 B, C3 1,048,576 mixed, C4 262,144 x 9000 B IPv6) through the default launch path, every
    packet's result word equal to the oracle's (the bench's oracle gate, as a test)."""
    import torch
    sid, n, stride = {"c1": (O.SYNTH_C1, 1 << 20, 64), "c2": (O.SYNTH_C2, 1 << 20, 2048),
                      "c3": (O.SYNTH_C3, 1 << 20, 2048), "c4": (O.SYNTH_C4, 1 << 18, 9216)}[cfg]
    a, d = orc.synth(n, stride, 0, sid, O.SEED, 0)
    want, want_st = orc.process(a, d, threads=8)
    arena = torch.from_numpy(a).pin_memory().cuda()
    dt = V.desc_to_tensor(d)
    del a
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.compute(arena, dt, n, out, st, O.MODE_COMPUTE)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(st.cpu().numpy(), want_st)
    # the sums written into the frames, then verified: every requested sum checks out
    V.compute(arena, dt, n, out, None, O.MODE_WRITE)
    V.compute(arena, dt, n, None, st, O.MODE_VERIFY)
    torch.cuda.synchronize()
    want_ok = np.where(d["flags"] & O.F_IP, O.S_IP_OK, 0) | np.where(d["flags"] & O.F_L4, O.S_L4_OK, 0)
    assert np.array_equal(st.cpu().numpy() & (O.S_IP_OK | O.S_L4_OK), want_ok.astype(np.uint8))
    del arena
    torch.cuda.empty_cache()


@pytest.mark.parametrize("team", [0, 3, 9, 40, 45, 46, 47])
def test_packet_ending_at_unaligned_arena_end(V, orc, team):
    """Arena length not a multiple of 16 and the last packet ending exactly at the arena end:
    the final partial chunk must still be read (buffer-descriptor range rounding)."""
    kats, frames, infos = kat_batch()
    for fr, inf in zip(frames, infos):
        for pad in (0, 1, 5, 14):
            arena = np.zeros(pad + len(fr), np.uint8)
            arena[pad:] = np.frombuffer(fr, np.uint8)
            rows = [(pad + x.l3_off, x.l3_len, x.l4_off, x.ver, x.proto, O.desc_flags_for(x), 0) for x in inf]
            desc = np.array(rows, dtype=O.DESC_DTYPE)
            out, st, _ = gpu_compute(V, arena, desc, O.MODE_VERIFY, team)
            oout, ost = orc.process(arena, desc, O.MODE_VERIFY)
            assert np.array_equal(out, oout) and np.array_equal(st, ost), (pad, len(fr))


def test_context_sparse_gather_and_zero_copy(V, orc):
    """Few packets scattered over a large arena: the pageable path gathers only touched blocks;
    the registered path runs zero-copy (kernel on the host frames, in-place writes)."""
    big = np.zeros(64 << 20, np.uint8)
    a_small, d_small = orc.synth(300, 2048, 14, O.SYNTH_FUZZ, O.SEED, 4242)
    rng = np.random.default_rng(3)
    slots = np.sort(rng.choice((64 << 20) // 9216 - 1, 300, replace=False))
    desc = d_small.copy()
    for i, sl in enumerate(slots):
        big[sl * 9216: sl * 9216 + 2048] = a_small[i * 2048:(i + 1) * 2048]
        desc[i]["l3_off"] = sl * 9216 + 14
    want_out, want_st = orc.process(big, desc, O.MODE_COMPUTE)
    ctx = V.Context(0, max_arena=1 << 22, max_pkts=1024)     # far smaller than the span
    out, st = ctx.run(big, desc)
    assert np.array_equal(out, want_out) and np.array_equal(st, want_st)
    # zero-copy on the registered arena, with in-place writes
    want_arena = big.copy()
    orc.process(want_arena, desc, O.MODE_COMPUTE, write=True)
    ctx.register(big)
    out2 = np.zeros(len(desc), np.uint32)
    ctx.wait(ctx.submit(big, desc, out2, None, O.MODE_WRITE))
    assert np.array_equal(out2, want_out)
    assert np.array_equal(big, want_arena)
    out3, st3 = ctx.run(big, desc, O.MODE_VERIFY)
    assert np.all(st3 & O.S_L4_OK)
    ctx.close()


def test_egress_batch_mirror(V, orc):
    """vswitch seam: NAT-style rewrites on the CPU mark sums dirty (setters + checksumSkipped),
    EgressBatch defers them and flushes once at completeTx; frames must equal Java's full
    recompute (oracle)."""
    from vproxy_amd import vswitch as S
    n, stride = 2000, 2048
    arena, desc = orc.synth(n, stride, 14, O.SYNTH_C3, O.SEED, 99)
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)          # valid input checksums
    rng = np.random.default_rng(8)
    batch = S.EgressBatch(arena, capacity=256)
    want = arena.copy()
    for i in range(n):
        d = desc[i]
        l3 = int(d["l3_off"])
        kind = rng.integers(0, 4)
        ip_dirty = l4_dirty = False
        if kind == 1:      # setSrc -> IP dirty + pseudoHeaderChanges (TCP/UDP)
            new = rng.integers(0, 256, 4, dtype=np.uint8)
            arena[l3 + 12:l3 + 16] = new
            want[l3 + 12:l3 + 16] = new
            ip_dirty = True
            l4_dirty = int(d["l4_proto"]) in (6, 17)
        elif kind == 2:    # TTL decrement (IPInputRoute) -> IP dirty
            arena[l3 + 8] -= 1
            want[l3 + 8] -= 1
            ip_dirty = True
        elif kind == 3 and int(d["l4_proto"]) in (6, 17):   # setDstPort -> L4 dirty
            arena[l3 + 22:l3 + 24] = [0, 121]
            want[l3 + 22:l3 + 24] = [0, 121]
            l4_dirty = True
        f = S.checksum_flags_for(True, ip_dirty, int(d["l4_proto"]), l4_dirty)
        if f:
            one = desc[i:i + 1].copy()
            one["flags"] = f
            orc.process(want, one, O.MODE_COMPUTE, write=True)
        batch.defer(l3, int(d["l3_len"]), int(d["l4_off"]), 4, int(d["l4_proto"]), f)
    batch.complete_tx()
    assert batch.stats["tx_csum_gpu"] > 0
    assert np.array_equal(arena, want)
    batch.close()


def test_cpp_consumer_runs(V, tmp_path):
    """Run the plain-C++ C-ABI consumer (ctx API + PNI entry points) on the GPU."""
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "capi_smoke"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", os.path.join(repo, "include"),
                           os.path.join(repo, "tests", "cpp", "capi_smoke.cpp"), "-L", os.path.join(repo, "vproxy_amd"),
                           "-lvpcsum", "-Wl,-rpath," + os.path.join(repo, "vproxy_amd"), "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi ok" in r.stdout


# ---- K2 grids: grid-stride over 64-packet units at any workgroup count ----

@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4097, 40000])
@pytest.mark.parametrize("bpc", [0, 1, 2, 5])
def test_grids(V, orc, n, bpc):
    """Ragged C3 batches vs oracle: partial last units, waves without a unit, 1-12 workgroups
    per CU; repeated back to back on one stream."""
    import torch
    a, d = orc.synth(n, 2048, 0, O.SYNTH_C3, O.SEED, 777 + n)
    want, want_st = orc.process(a, d)
    arena = dev(a)
    dt = V.desc_to_tensor(d)
    for rep in range(2):
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        st = torch.zeros(n, dtype=torch.uint8, device="cuda")
        V.compute(arena, dt, n, out, st, O.MODE_COMPUTE, 0, blocks_per_cu=bpc)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want), (n, bpc, rep)
        assert np.array_equal(st.cpu().numpy(), want_st), (n, bpc, rep)


def test_small_grids(V, orc):
    """Grids of 1..9 workgroups (the launcher caps the grid at ceil(m / 256) workgroups, so a
    batch of m = 256 g packets at one workgroup per CU runs on exactly g workgroups): every
    unit is done once and nothing past the batch is written."""
    import torch
    n = 64 * 53 + 17
    a, d = orc.synth(n, 2048, 0, O.SYNTH_C3, O.SEED, 4242)
    want, _ = orc.process(a, d)
    arena = dev(a)
    dt = V.desc_to_tensor(d)
    for g in range(1, 10):
        out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        m = min(n, 256 * g)
        V.compute(arena, dt, m, out, None, O.MODE_COMPUTE, 0, blocks_per_cu=1)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert np.array_equal(got[:m], want[:m]), g
        assert np.all(got[m:] == 0xFFFFFFFF), g


def test_two_streams_concurrent(V, orc):
    """Launches on two streams run concurrently and share no state."""
    import torch
    n = 50000
    a, d = orc.synth(n, 2048, 0, O.SYNTH_C2, O.SEED, 99)
    want, _ = orc.process(a, d)
    arena = dev(a)
    dt = V.desc_to_tensor(d)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(8)]
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        V.compute(arena, dt, n, o, None, O.MODE_COMPUTE, 0, stream=(s1 if i % 2 else s2))
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint32), want)


def test_low_concurrency_grid(V, orc):
    """The sampled low-concurrency grid (all 64 sampled descriptors >= 1 KiB -> 2 workgroups per
    CU) covers every packet, including small ones the sample did not see."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = cus * 2 * 256 + 9000          # more packets than the low grid holds in one round
    a, d = orc.synth(n, 2048, 0, O.SYNTH_C2, O.SEED, 5)
    sampled = {(n * lane) >> 6 for lane in range(64)}
    small = np.array([i for i in range(3, n, 7) if i not in sampled])
    d = d.copy()
    d["l3_len"][small] = 64            # descriptors define the range; the oracle follows them too
    want, want_st = orc.process(a, d, O.MODE_VERIFY)
    arena = dev(a)
    dt = V.desc_to_tensor(d)
    for full in (False, True):
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        st = torch.zeros(n, dtype=torch.uint8, device="cuda")
        V.compute(arena, dt, n, out, st, O.MODE_VERIFY, 0, full_grid=full)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want), full
        assert np.array_equal(st.cpu().numpy(), want_st), full


def test_staged_result_stores(V, orc):
    """Large-packet batches big enough that every wave of the low-concurrency grid takes >= 4
    units stage their out / status words in LDS: n is not a multiple of 64
    (a partial last unit), some descriptors are bad, some packets small, one raw range; verify
    mode (out + status), compute mode (out only), and write mode (checksum fields in place, the
    words staged) all equal the oracle's, and the default equals variant 76 (no staging)."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = 4 * (cus * 2 * 256) + 9000 + 37          # >= 4 units per wave of the 2-WG/CU grid
    a, d = orc.synth(n, 2048, 0, O.SYNTH_C2, O.SEED, 77)
    sampled = {(n * lane) >> 6 for lane in range(64)}
    rng = np.random.default_rng(77)
    pick = np.array(sorted(set(rng.choice(n, 4000, replace=False).tolist()) - sampled))
    d = d.copy()
    d["l3_len"][pick[:1500]] = 64                  # small packets the sample did not see
    d["l3_len"][pick[1500:2000]] = 0               # bad: shorter than an IPv4 header
    d["l3_off"][pick[2000:2300]] = a.size + 4096   # bad: outside the arena
    d["flags"][pick[2300:2400]] = O.F_RAW          # raw ranges
    want, want_st = orc.process(a, d, O.MODE_VERIFY, threads=8)
    arena = dev(a)
    dt = V.desc_to_tensor(d)
    for team in (0, 76):
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        st = torch.zeros(n, dtype=torch.uint8, device="cuda")
        V.compute(arena, dt, n, out, st, O.MODE_VERIFY, team)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want), team
        assert np.array_equal(st.cpu().numpy(), want_st), team
        out.zero_()
        V.compute(arena, dt, n, out, None, O.MODE_COMPUTE, team)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want), team
    # write mode: the fields land in the frames (direct stores), the words are staged
    w_out, _ = orc.process(a, d, O.MODE_COMPUTE, write=True)   # a now holds the written frames
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    V.compute(arena, dt, n, out, None, O.MODE_WRITE, 0)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), w_out)
    assert np.array_equal(arena.cpu().numpy(), a)


@pytest.mark.parametrize("cfg", ["c1", "c3"])
def test_status_bytes_at_any_alignment(V, orc, cfg):
    """Status bytes of whole units go out as one dword per 4 packets when the unit's bytes start
    4-B aligned, as bytes otherwise (K2 store_result PACK): a status buffer at offsets 0..3 of a
    larger one, window units (C1 dense frames) and the team path (C3), a partial last unit.  Every
    byte equals the oracle's and nothing outside [off, off + n) is written."""
    import torch
    sid, stride = {"c1": (O.SYNTH_C1, 64), "c3": (O.SYNTH_C3, 2048)}[cfg]
    n = 20_000 + 37
    a, d = orc.synth(n, stride, 0, sid, O.SEED, 7)
    d = d.copy()
    d["l3_len"][100:164:3] = 0                     # bad descriptors inside a few units
    want, want_st = orc.process(a, d, O.MODE_VERIFY, threads=8)
    arena = dev(a)
    dt = V.desc_to_tensor(d)
    for off in range(4):
        buf = torch.full((n + 8,), 0xEE, dtype=torch.uint8, device="cuda")
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        V.compute(arena, dt, n, out, buf[off:off + n], O.MODE_VERIFY)
        torch.cuda.synchronize()
        b = buf.cpu().numpy()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want), off
        assert np.array_equal(b[off:off + n], want_st), off
        assert (b[:off] == 0xEE).all() and (b[off + n:] == 0xEE).all(), off


@pytest.mark.parametrize("team", [0, 84])
def test_workgroup_sorted_units(V, orc, team):
    """Mixed batches large enough for the sampled grid, where the 4 waves of a workgroup rank
    their 256 packets by cost class together (the default, and variant 84):
    C3 packets with bad descriptors, raw ranges, runs of small packets of one shape (window-unit
    candidates, which workgroup-sorted units do not take), n not a multiple of 256 (waves past the
    batch in the last workgroup) and more units than one grid-stride round.  Verify, compute and
    write modes equal the oracle's, and variant 76 (per-wave units) equals both."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = cus * 12 * 256 + 100_000 + 37            # a second grid-stride round for some workgroups
    a, d = orc.synth(n, 2048, 0, O.SYNTH_C3, O.SEED, 84)
    sampled = {(n * lane) >> 6 for lane in range(64)}
    rng = np.random.default_rng(84)
    pick = np.array(sorted(set(rng.choice(n, 6000, replace=False).tolist()) - sampled))
    d = d.copy()
    d["l3_len"][pick[:500]] = 0                    # bad: shorter than an IPv4 header
    d["l3_off"][pick[500:800]] = a.size + 4096     # bad: outside the arena
    d["flags"][pick[800:900]] = O.F_RAW            # raw ranges
    # units of 64 packets of one small shape (window units in per-wave mode): C3's own 64-B
    # IPv4/UDP packets copied over whole units
    small = np.flatnonzero((d["l3_len"] == 64) & (d["l3_ver"] == 4) & (d["l4_proto"] == 17))
    src = int(small[0])
    for u in (1000, 1001, 2500):
        for i in range(u * 64, u * 64 + 64):
            a[i * 2048:(i + 1) * 2048] = a[src * 2048:(src + 1) * 2048]
            d[i] = d[src]
            d["l3_off"][i] = d["l3_off"][src] - src * 2048 + i * 2048
    want, want_st = orc.process(a, d, O.MODE_VERIFY, threads=8)
    arena = dev(a)
    dt = V.desc_to_tensor(d)
    for v in (team, 76):
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        st = torch.zeros(n, dtype=torch.uint8, device="cuda")
        V.compute(arena, dt, n, out, st, O.MODE_VERIFY, v)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want), v
        assert np.array_equal(st.cpu().numpy(), want_st), v
        out.zero_()
        V.compute(arena, dt, n, out, None, O.MODE_COMPUTE, v)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want), v
    w_out, _ = orc.process(a, d, O.MODE_COMPUTE, write=True)   # a now holds the written frames
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    V.compute(arena, dt, n, out, None, O.MODE_WRITE, team)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), w_out)
    assert np.array_equal(arena.cpu().numpy(), a)
    # the frames now hold their sums: verify reports every requested one as correct
    V.compute(arena, dt, n, None, st, O.MODE_VERIFY, team)
    torch.cuda.synchronize()
    ok = np.where(d["flags"] & O.F_IP, O.S_IP_OK, 0) | np.where(d["flags"] & O.F_L4, O.S_L4_OK, 0)
    sel = ((want_st & O.S_DONE) != 0) & ((d["flags"] & O.F_RAW) == 0)
    assert np.array_equal(st.cpu().numpy()[sel] & (O.S_IP_OK | O.S_L4_OK), ok.astype(np.uint8)[sel])


# ---- low-latency service (persistent grid polling a pinned mailbox) ----

def _busy_us(us):
    import time
    t = time.perf_counter() + us * 1e-6
    while time.perf_counter() < t:
        pass


@pytest.mark.parametrize("idle_us", [5000, 40])
def test_service_flushes(V, orc, idle_us):
    """Flushes from a registered arena through the service: bit-exact with the oracle over
    consecutive batches of random sizes in all three modes.  With idle_us = 40 the grid leaves
    between most flushes, some of them while a batch is being posted; the host restarts it and
    re-runs a batch a leaving grid did not finish."""
    n_all, stride = 4096, 9216          # frames must not overlap: WRITE mode stores into them
    a, d = orc.synth(n_all, stride, 14, O.SYNTH_FUZZ, O.SEED, 31 + idle_us)
    arena = np.zeros(a.size + 4096, np.uint8)
    arena[:a.size] = a
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=n_all)
    ctx.register(arena)
    ctx.set_service(idle_us)
    rng = np.random.default_rng(idle_us)
    iters = 90
    for it in range(iters):
        lo = int(rng.integers(0, n_all - 1))
        b = int(rng.integers(1, min(512, n_all - lo) + 1))     # <= the service's batch limit
        dsc = d[lo:lo + b].copy()
        mode = (O.MODE_COMPUTE, O.MODE_VERIFY, O.MODE_WRITE)[it % 3]
        if it % 10 == 5:   # the host rewrites frame bytes between flushes: no stale reads
            arena[int(dsc[0]["l3_off"]) + 30:int(dsc[0]["l3_off"]) + 60] ^= np.uint8(0x5A)
        want_arena = arena.copy()
        want_out, want_st = orc.process(want_arena, dsc, mode & O.MODE_VERIFY, write=bool(mode & O.MODE_WRITE))
        out = np.zeros(b, np.uint32)
        st = np.zeros(b, np.uint8)
        ctx.wait(ctx.submit(arena, dsc, out, st, mode))
        assert np.array_equal(out, want_out), it
        assert np.array_equal(st, want_st), it
        assert np.array_equal(arena, want_arena), it
        _busy_us(int(rng.integers(0, 3 * idle_us)))
    s = ctx.stats()
    assert s["service_batches"] == iters
    assert s["service_launches"] >= 1
    # two flushes in flight: the second submit hands the first one's results over first
    want_all, _ = orc.process(arena, d)
    o1, o2 = np.zeros(300, np.uint32), np.zeros(200, np.uint32)
    t1 = ctx.submit(arena, d[:300], o1)
    t2 = ctx.submit(arena, d[300:500], o2)
    ctx.wait(t2)
    ctx.wait(t1)
    assert np.array_equal(np.concatenate([o1, o2]), want_all[:500])
    # a batch above the service's limit is launched as usual
    o3 = np.zeros(n_all, np.uint32)
    ctx.wait(ctx.submit(arena, d, o3))
    assert np.array_equal(o3, want_all)
    assert ctx.stats()["service_batches"] == iters + 2
    ctx.set_service(0)
    o4 = np.zeros(100, np.uint32)
    ctx.wait(ctx.submit(arena, d[:100], o4))
    assert np.array_equal(o4, want_all[:100])
    assert ctx.stats()["service_batches"] == iters + 2
    ctx.close()


@pytest.mark.parametrize("idle_us", [20000, 30])
def test_service_inline_flushes(V, orc, idle_us):
    """Flushes of 1..3 frames take their descriptors from the command's mailbox line (tagged
    with the batch's low sequence byte); 4-frame flushes interleave and read the descriptor
    buffer.  600 flushes wrap the tag byte twice; descriptors include rejected ones (FUZZ), and
    consecutive flushes reuse the same inline slots with different descriptors and modes."""
    n_all, stride = 128, 9216          # frames must not overlap: WRITE mode stores into them
    a, d = orc.synth(n_all, stride, 14, O.SYNTH_FUZZ, O.SEED, 77 + idle_us)
    arena = np.zeros(a.size + 4096, np.uint8)
    arena[:a.size] = a
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=n_all)
    ctx.register(arena)
    ctx.set_service(idle_us)
    rng = np.random.default_rng(idle_us + 1)
    iters = 600
    for it in range(iters):
        b = 4 if it % 7 == 3 else int(rng.integers(1, 4))
        idx = rng.choice(n_all, size=b, replace=False)
        dsc = d[idx].copy()
        mode = (O.MODE_COMPUTE, O.MODE_VERIFY, O.MODE_WRITE)[int(rng.integers(0, 3))]
        want_arena = arena.copy()
        want_out, want_st = orc.process(want_arena, dsc, mode & O.MODE_VERIFY, write=bool(mode & O.MODE_WRITE))
        out = np.zeros(b, np.uint32)
        st = np.zeros(b, np.uint8)
        ctx.wait(ctx.submit(arena, dsc, out, st, mode))
        assert np.array_equal(out, want_out), it
        assert np.array_equal(st, want_st), it
        assert np.array_equal(arena, want_arena), it
        if idle_us < 100 and it % 5 == 0:
            _busy_us(int(rng.integers(0, 3 * idle_us)))
    assert ctx.stats()["service_batches"] == iters
    ctx.close()


def test_service_egress_batch(V, orc):
    """EgressBatch with the service: same frames as Java's full recompute after TTL rewrites."""
    from vproxy_amd import vswitch as S
    n, stride = 600, 2048
    arena, desc = orc.synth(n, stride, 14, O.SYNTH_C3, O.SEED, 7)
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)
    want = arena.copy()
    batch = S.EgressBatch(arena, capacity=128, service_idle_us=20000)
    for i in range(n):
        l3 = int(desc[i]["l3_off"])
        arena[l3 + 8] -= 1
        want[l3 + 8] -= 1
        one = desc[i:i + 1].copy()
        one["flags"] = O.F_IP
        orc.process(want, one, O.MODE_COMPUTE, write=True)
        batch.defer(l3, int(desc[i]["l3_len"]), int(desc[i]["l4_off"]), 4, int(desc[i]["l4_proto"]), O.F_IP)
    batch.complete_tx()
    assert np.array_equal(arena, want)
    assert batch.ctx.stats()["service_batches"] == batch.stats["flushes"] >= 5
    batch.close()


def test_verify_frames_rx_batch(V, orc):
    """Ingress verify of a received batch (ctx_verify_frames): raw Ethernet frames in a registered
    arena are parsed and verified on the GPU; status and sums must equal the Java parse rules
    (oracle parse_ether) followed by the oracle's verify, frame for frame."""
    frames = []
    for fn in sorted(os.listdir(os.path.join(GOLD, "pcap"))):
        lt, pkts = read_pcap(os.path.join(GOLD, "pcap", fn))
        if lt == 1:
            frames += pkts
    kats = json.load(open(os.path.join(GOLD, "kat.json")))["kats"]
    frames += [bytes.fromhex(k["hex"]) for k in kats if k["layer"] == "ether"]
    base = bytes.fromhex(kats[2]["hex"])
    frames.append(base[:12] + b"\x81\x00\x00\x05" + base[12:])   # VLAN
    frames.append(base[:30])                                     # truncated
    frames.append(base[:12] + b"\x08\x06" + base[14:])           # ARP
    # synthetic frames: C3 / C5 / FUZZ L3 packets behind an Ethernet header, valid and corrupted sums
    rng = np.random.default_rng(12)
    for wl in (O.SYNTH_C3, O.SYNTH_C5, O.SYNTH_FUZZ):
        a, d = orc.synth(300, 9216, 14, wl, O.SEED, 50 + wl)
        orc.process(a, d, O.MODE_COMPUTE, write=True)
        for i in range(len(d)):
            o, L = int(d[i]["l3_off"]), int(d[i]["l3_len"])
            eth = bytearray(14)
            eth[12:14] = b"\x08\x00" if d[i]["l3_ver"] == 4 else b"\x86\xdd"
            f = bytearray(eth + bytes(a[o:o + L]))
            if rng.random() < 0.2:
                f[14 + L // 2] ^= 0xA5
            frames.append(bytes(f))
    offs, lens, arena = [], [], bytearray()
    for f in frames:
        arena += bytes(int(rng.integers(0, 64)))                 # any alignment
        offs.append(len(arena))
        lens.append(len(f))
        arena += f
    arena = np.frombuffer(bytes(arena) + bytes(4096), np.uint8).copy()
    want_st = np.zeros(len(frames), np.uint8)
    want_out = np.zeros(len(frames), np.uint32)
    for i, f in enumerate(frames):
        info, _ = O.parse_ether(f)
        if info is None:
            want_st[i] = O.S_BAD_DESC
            continue
        one = np.array([(offs[i] + info.l3_off, info.l3_len, info.l4_off, info.ver, info.proto,
                         O.desc_flags_for(info), 0)], dtype=O.DESC_DTYPE)
        o, st = orc.process(arena, one, O.MODE_VERIFY)
        want_out[i], want_st[i] = o[0], st[0]
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=4096)
    ctx.register(arena)
    before = arena.copy()
    out, st = ctx.verify_frames(arena, np.array(offs), np.array(lens))
    assert np.array_equal(st, want_st)
    ok = (want_st & O.S_BAD_DESC) == 0
    assert np.array_equal(out[ok], want_out[ok])
    assert np.array_equal(arena, before)                         # verify never writes frames
    assert int(np.sum(ok)) > 900 and int(np.sum((st & O.S_L4_OK) == 0)) > 100
    # the seam's form (GpuCsumBatch.verifyFrames): no out words, the same status bytes
    none, st2 = ctx.verify_frames(arena, np.array(offs), np.array(lens), sums=False)
    assert none is None and np.array_equal(st2, want_st)
    # and the descriptor form without out words, staged (a pageable copy) and zero-copy
    infos = [O.parse_ether(f)[0] for f in frames]
    dd = np.array([(offs[i] + x.l3_off, x.l3_len, x.l4_off, x.ver, x.proto, O.desc_flags_for(x), 0)
                   for i, x in enumerate(infos) if x is not None], dtype=O.DESC_DTYPE)
    for a in (arena, arena.copy()):
        st3 = np.zeros(len(dd), np.uint8)
        ctx.wait(ctx.submit(a, dd, None, st3, O.MODE_VERIFY))
        assert np.array_equal(st3, want_st[ok])
    # RX batches of up to 512 frames on the service grid (parse + verify per frame, no launch), with
    # and without out words
    ctx.set_service(20000)
    offs_a, lens_a = np.array(offs), np.array(lens)
    for lo in range(0, len(frames), 400):
        sl = slice(lo, min(lo + 400, len(frames)))
        out4, st4 = ctx.verify_frames(arena, offs_a[sl], lens_a[sl])
        assert np.array_equal(st4, want_st[sl]), lo
        ok4 = (want_st[sl] & O.S_BAD_DESC) == 0
        assert np.array_equal(out4[ok4], want_out[sl][ok4]), lo
        _, st5 = ctx.verify_frames(arena, offs_a[sl], lens_a[sl], sums=False)
        assert np.array_equal(st5, want_st[sl]), lo
    assert ctx.stats()["service_batches"] == 2 * ((len(frames) + 399) // 400)
    assert np.array_equal(arena, before)
    ctx.close()


# ---- checksum offload: pseudo-header partial sums (VPCSUM_F_L4P, VP_CSUM_UP_PSEUDO) ----

@pytest.mark.parametrize("team", [0, 2, 6, 40, 45, 46, 47, 62])
@pytest.mark.parametrize("workload", [O.SYNTH_C3, O.SYNTH_C4, O.SYNTH_FUZZ])
def test_l4_pseudo_partial(V, orc, team, workload):
    """F_L4P on every packet (with and without F_IP), all modes, against the oracle: the field
    gets the folded pseudo-header sum (CHECKSUM_PARTIAL); ICMPv4 and F_L4P|F_L4 are rejected."""
    stride = 9216
    n = 700
    arena, desc = orc.synth(n, stride, 5, workload, O.SEED, 90 + workload)
    rng = np.random.default_rng(workload)
    desc = desc.copy()
    f = np.where(desc["l3_ver"] == 4, O.F_IP, 0) | O.F_L4P
    f[rng.random(n) < 0.1] |= O.F_L4        # invalid combination -> BAD
    f[rng.random(n) < 0.2] &= ~O.F_IP
    desc["flags"] = f
    for mode, write in ((O.MODE_COMPUTE, False), (O.MODE_VERIFY, False), (O.MODE_COMPUTE, True)):
        out, st, after = gpu_compute(V, arena, desc, mode, team, write=write)
        a2 = arena.copy()
        oout, ost = orc.process(a2, desc, mode, write=write)
        assert np.array_equal(st, ost), (mode, write)
        assert np.array_equal(out, oout), (mode, write)
        if write:
            assert np.array_equal(after, a2)
    # after WRITE every F_L4P packet verifies as partial
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)
    _, st, _ = gpu_compute(V, arena, desc, O.MODE_VERIFY, team)
    good = (st & O.S_BAD_DESC) == 0
    assert np.all(st[good] & O.S_L4_OK)


def test_l4_pseudo_partial_pcap(V, orc):
    """The reference's CHECKSUM_PARTIAL pcap frames verify under F_L4P on the GPU."""
    partial = 0
    for fn in sorted(os.listdir(os.path.join(GOLD, "pcap"))):
        lt, pkts = read_pcap(os.path.join(GOLD, "pcap", fn))
        for p in pkts:
            off = l3_offset(lt, p)
            if off is None:
                continue
            info, err = O.parse_l3(p, off, len(p) - off)
            if info is None or info.proto != O.IP_PROTOCOL_TCP:
                continue
            arena = np.frombuffer(p + bytes(64), np.uint8).copy()
            desc = np.array([(off, info.l3_len, info.l4_off, info.ver, info.proto, O.F_L4, 0),
                             (off, info.l3_len, info.l4_off, info.ver, info.proto, O.F_L4P, 0)], dtype=O.DESC_DTYPE)
            out, st, _ = gpu_compute(V, arena, desc, O.MODE_VERIFY)
            oout, ost = orc.process(arena, desc, O.MODE_VERIFY)
            assert np.array_equal(out, oout) and np.array_equal(st, ost)
            if not st[0] & O.S_L4_OK:
                assert st[1] & O.S_L4_OK
                partial += 1
    assert partial == 12


@pytest.mark.parametrize("order", ["sorted", "shuffled"])
def test_arena_beyond_4gib(V, orc, order):
    """Arenas past the 32-bit buffer-descriptor range (> 4 GiB, as a umem of a large switch can
    be): packets below and above 4 GiB, in address order and shuffled across the whole 5 GiB, go
    through the team kernel's 64-bit loads, bit-exact."""
    variant = 0
    import torch
    n, stride = 1500, 9216                                     # FUZZ frames reach 9000 B
    a, d = orc.synth(n, stride, 6, O.SYNTH_FUZZ, O.SEED, 4444)
    want, want_st = orc.process(a, d, O.MODE_VERIFY)
    big = torch.zeros((5 << 30) + 4096, dtype=torch.uint8, device="cuda")
    rng = np.random.default_rng(4)
    bases = np.sort(rng.choice(((5 << 30) - (1 << 20)) // 16384, n, replace=False)) * 16384 + 8
    bases[: n // 3] = np.arange(n // 3) * 16384 + 8          # a third below 4 GiB
    if order == "shuffled":
        rng.shuffle(bases)
    dg = d.copy()
    src = torch.from_numpy(a).pin_memory().cuda()
    for i in range(n):
        big[int(bases[i]): int(bases[i]) + stride] = src[i * stride:(i + 1) * stride]
        dg[i]["l3_off"] = int(bases[i]) + int(d[i]["l3_off"]) - i * stride
    assert int(dg["l3_off"].max()) > (4 << 30)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    dt = V.desc_to_tensor(dg)
    V.compute(big, dt, n, out, st, O.MODE_VERIFY, variant)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(st.cpu().numpy(), want_st)
    # in-place writes land at the right > 4 GiB addresses
    a2 = a.copy()
    orc.process(a2, d, O.MODE_COMPUTE, write=True)
    V.compute(big, dt, n, out, None, O.MODE_WRITE, variant)
    torch.cuda.synchronize()
    for i in rng.choice(n, 64, replace=False):
        got = big[int(bases[i]): int(bases[i]) + stride].cpu().numpy()
        assert np.array_equal(got, a2[i * stride:(i + 1) * stride]), i
    del big
    torch.cuda.empty_cache()


def test_batches_straddling_4gib(V, orc):
    """Dense 64-B frames and C2 frames of one batch straddling the 4-GiB line of a large arena
    (the team kernel's 64-bit loads), bit-exact with the oracle in compute,
    verify and write-back."""
    variant = 0
    import torch
    base = (4 << 30) - (64 << 10)
    for sid, m, stride, pad in ((O.SYNTH_C1, 4096 + 37, 64, 14), (O.SYNTH_C2, 700, 2048, 0)):
        a, d = orc.synth(m, stride, pad, sid, O.SEED, 77)
        want, want_st = orc.process(a, d, O.MODE_COMPUTE)
        big = torch.zeros(base + len(a) + 4096, dtype=torch.uint8, device="cuda")
        big[base:base + len(a)] = torch.from_numpy(a).pin_memory().cuda()
        dg = d.copy()
        dg["l3_off"] += base
        assert int(dg["l3_off"].min()) < (4 << 30) < int(dg["l3_off"].max())
        dt = V.desc_to_tensor(dg)
        out = torch.zeros(m, dtype=torch.int32, device="cuda")
        st = torch.zeros(m, dtype=torch.uint8, device="cuda")
        V.compute(big, dt, m, out, st, O.MODE_COMPUTE, variant)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
        assert np.array_equal(st.cpu().numpy(), want_st)
        a2 = a.copy()
        orc.process(a2, d, O.MODE_COMPUTE, write=True)
        V.compute(big, dt, m, out, None, O.MODE_WRITE, variant)
        torch.cuda.synchronize()
        assert np.array_equal(big[base:base + len(a)].cpu().numpy(), a2)
        V.compute(big, dt, m, out, st, O.MODE_VERIFY, variant)
        torch.cuda.synchronize()
        vo, vs = orc.process(a2.copy(), d, O.MODE_VERIFY)
        assert np.array_equal(st.cpu().numpy(), vs)
        del big
        torch.cuda.empty_cache()


@pytest.mark.parametrize("order", ["sorted", "reversed", "two_swapped"])
def test_windowed_k2_past_4gib(V, orc, order):
    """The default launcher on a 9-GiB arena runs K2 once per 2-GiB window (kernels.hip kWinBytes):
    dense 64-B frames straddling the 2-GiB and 4-GiB window lines, C2 frames in the fourth window,
    mixed FUZZ frames at the arena's end (the window [8, 9) GiB is cut short by the arena end).  Sorted descriptors go to their
    windows' launches; reversed ones and a batch with two descriptors swapped across windows leave
    packets to the leftover pass (k_win_left).  Compute, verify and write-back equal the oracle."""
    import torch
    pieces = []   # (synth id, packets, stride, pad, arena offset)
    pieces.append((O.SYNTH_C1, 3000, 64, 14, (2 << 30) - 64 * 1500))
    pieces.append((O.SYNTH_C1, 3000, 64, 14, (4 << 30) - 64 * 1500))
    pieces.append((O.SYNTH_C2, 600, 2048, 0, (6 << 30) + 12345 * 16))
    pieces.append((O.SYNTH_FUZZ, 300, 9216, 6, (9 << 30) - 300 * 9216 - 4096))
    big = torch.zeros((9 << 30) + 64, dtype=torch.uint8, device="cuda")
    arrs, descs, wants = [], [], []
    for k, (sid, m, stride, pad, base) in enumerate(pieces):
        a, d = orc.synth(m, stride, pad, sid, O.SEED, 1000 * k)
        w, _ = orc.process(a, d, O.MODE_COMPUTE)
        big[base:base + len(a)] = torch.from_numpy(a).pin_memory().cuda()
        dg = d.copy()
        dg["l3_off"] += base
        arrs.append((base, a, d))
        descs.append(dg)
        wants.append(w)
    dall, want = np.concatenate(descs), np.concatenate(wants)
    perm = np.arange(len(dall))
    if order == "reversed":
        perm = perm[::-1].copy()
    elif order == "two_swapped":
        perm[[10, len(perm) - 10]] = perm[[len(perm) - 10, 10]]
    dall, want = dall[perm], want[perm]
    n = len(dall)
    dt = V.desc_to_tensor(dall)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.compute(big, dt, n, out, st, O.MODE_COMPUTE)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    assert np.all(st.cpu().numpy() == O.S_DONE)
    V.compute(big, dt, n, out, None, O.MODE_WRITE)
    V.compute(big, dt, n, None, st, O.MODE_VERIFY)
    torch.cuda.synchronize()
    stn = st.cpu().numpy()
    want_ok = np.where(dall["flags"] & 1, 1, 0) | np.where(dall["flags"] & 2, 2, 0)
    assert np.array_equal(stn & 3, want_ok)
    for base, a, d in arrs:
        a2 = a.copy()
        orc.process(a2, d, O.MODE_COMPUTE, write=True)
        assert np.array_equal(big[base:base + len(a)].cpu().numpy(), a2)
    del big
    torch.cuda.empty_cache()


@pytest.mark.parametrize("service", [False, True])
def test_parse_rules_on_gpu(V, orc, service):
    """k_parse_ether and ctx_verify_frames against the oracle's parse on frames at every edge of
    the reference's parse rules (tests/edgevec.py:parse_cases): TCP under 20 B, UDP under 8 B,
    empty ICMP, the version nibble not read by initPartial, the full Ipv6Packet.from behind an
    extension header (UDP length field, ICMP >= 8 B, TCP options), EtherIP, 802.1Q."""
    import torch
    import edgevec as E
    cases = E.parse_cases()
    offs, lens, arena = [], [], bytearray()
    for i, (f, _, _) in enumerate(cases):
        arena += bytes(i % 7)
        offs.append(len(arena))
        lens.append(len(f))
        arena += f
    arena = np.frombuffer(bytes(arena) + bytes(256), np.uint8).copy()
    n = len(cases)
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.parse_ether(dev(arena), dev(np.array(offs, np.uint64)), dev(np.array(lens, np.uint32)), n, d, st)
    torch.cuda.synchronize()
    got, stn = V.tensor_to_desc(d), st.cpu().numpy()
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
    ctx.register(arena)
    if service:   # the service grid parses each frame from its first 384 B staged in LDS
        ctx.set_service(20000)
    vout, vst = ctx.verify_frames(arena, np.array(offs), np.array(lens))
    assert ctx.stats()["service_batches"] == (1 if service else 0)
    ctx.close()
    for i, (f, ok, why) in enumerate(cases):
        info, err = O.parse_ether(f)
        assert (info is not None) == ok, why
        if info is None:
            assert stn[i] == O.S_BAD_DESC and vst[i] == O.S_BAD_DESC, why
            continue
        assert stn[i] == 0, why
        g = got[i]
        assert int(g["l3_off"]) == offs[i] + info.l3_off, why
        assert (g["l3_len"], g["l4_off"], g["l3_ver"], g["l4_proto"]) == (info.l3_len, info.l4_off, info.ver, info.proto), why
        assert g["flags"] == O.desc_flags_for(info), why
        one = np.array([(offs[i] + info.l3_off, info.l3_len, info.l4_off, info.ver, info.proto,
                         O.desc_flags_for(info), 0)], dtype=O.DESC_DTYPE)
        o, s = orc.process(arena, one, O.MODE_VERIFY)
        assert vst[i] == s[0] and vout[i] == o[0], why


@pytest.mark.parametrize("service", [0, 20000])
def test_unregister_with_batch_in_flight(V, orc, service):
    """Unregistering an arena while a zero-copy batch (launched, or on the service grid) still
    works on its frames finishes that batch first: the results are complete and the in-place
    writes landed; the next batch from the (now pageable) arena is staged."""
    n, stride = 300, 2048
    a, d = orc.synth(n, stride, 14, O.SYNTH_C3, O.SEED, 606)
    arena = np.concatenate([a, np.zeros(4096, np.uint8)])
    want_arena = arena.copy()
    want, _ = orc.process(want_arena, d, O.MODE_COMPUTE, write=True)
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
    ctx.register(arena)
    if service:
        ctx.set_service(service)
    out = np.zeros(n, np.uint32)
    t = ctx.submit(arena, d, out, None, O.MODE_WRITE)
    ctx.unregister(arena)
    ctx.wait(t)
    assert np.array_equal(out, want) and np.array_equal(arena, want_arena)
    out2, _ = ctx.run(arena, d)
    assert np.array_equal(out2, want)
    ctx.close()


def test_egress_small_flush_hand_back(V, orc):
    """GpuCsumBatch's SMALL_FLUSH rule in the mirror: a flush below the threshold goes back to the
    native path untouched (no GPU submit); from the threshold on it is computed on the GPU."""
    from vproxy_amd import vswitch as S
    n, stride = 12, 2048
    arena, desc = orc.synth(n, stride, 14, O.SYNTH_C3, O.SEED, 321)
    before = arena.copy()
    want = arena.copy()
    orc.process(want, desc[4:], O.MODE_COMPUTE, write=True)
    batch = S.EgressBatch(arena, capacity=64, small_flush=5)
    for d in desc[:4]:
        batch.defer(int(d["l3_off"]), int(d["l3_len"]), int(d["l4_off"]), 4, int(d["l4_proto"]), int(d["flags"]))
    assert batch.complete_tx() == 0 and np.array_equal(arena, before)
    assert len(batch.handed_back) == 1 and len(batch.handed_back[0]) == 4
    for d in desc[4:]:
        batch.defer(int(d["l3_off"]), int(d["l3_len"]), int(d["l4_off"]), 4, int(d["l4_proto"]), int(d["flags"]))
    assert batch.complete_tx() == 8 and np.array_equal(arena, want)
    batch.close()


def test_nat_arena_beyond_4gib(V, orc):
    """NAT on frames placed below and above 4 GiB of a 5-GiB arena (the 10M-packet C5 batch is a
    20-GB arena): the wide kernel addresses with 64-bit loads and stores, both entry formats."""
    import torch
    rng = np.random.default_rng(44)
    arena, desc, rw = _nat48_batch(orc, rng, 600, 6)
    n, stride = len(desc), 9088
    want = arena.copy()
    want_st = orc.nat_java(want, desc, rw)
    big = torch.zeros((5 << 30) + 4096, dtype=torch.uint8, device="cuda")
    bases = np.sort(rng.choice(((5 << 30) - (1 << 20)) // 16384, n, replace=False)) * 16384 + 8
    bases[: n // 3] = np.arange(n // 3) * 16384 + 8
    dg = desc.copy()
    src = torch.from_numpy(arena).pin_memory().cuda()
    for i in range(n):
        big[int(bases[i]): int(bases[i]) + stride] = src[i * stride:(i + 1) * stride]
        dg[i]["l3_off"] = int(bases[i]) + int(desc[i]["l3_off"]) - i * stride
    assert int(dg["l3_off"].max()) > (4 << 30)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.nat(big, V.desc_to_tensor(dg), dev(rw.view(np.uint8)), n, st, V.NAT_RFC1624)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), want_st)
    for i in rng.choice(n, 100, replace=False):
        got = big[int(bases[i]): int(bases[i]) + stride].cpu().numpy()
        assert np.array_equal(got, want[i * stride:(i + 1) * stride]), i
    del big
    torch.cuda.empty_cache()




def test_parse_tuples_match_oracle(V, orc):
    """vpcsum_parse_ether_tuples_async (batched header parse + flow tuple)
    against oracle.flow_tuple frame by frame: the reference's pcap and KAT frames, every edge frame
    of the parse rules (tests/edgevec.py:parse_cases), and 4000 fuzzed IPv4/IPv6 TCP/UDP/ICMP
    packets (options, IPv6 without extension headers) in Ethernet frames at odd offsets.  The
    descriptors equal those of the plain parse."""
    import torch
    import edgevec as E
    frames = [f for f, _, _ in E.parse_cases()]
    for fn in sorted(os.listdir(os.path.join(GOLD, "pcap"))):
        lt, pkts = read_pcap(os.path.join(GOLD, "pcap", fn))
        if lt == 1:
            frames += pkts
    kats = json.load(open(os.path.join(GOLD, "kat.json")))["kats"]
    frames += [bytes.fromhex(k["hex"]) for k in kats if k["layer"] == "ether"]
    a, d = orc.synth(4000, 2048, 14, O.SYNTH_FUZZ, O.SEED, 4242)
    for r in d:
        l3 = bytes(a[int(r["l3_off"]):int(r["l3_off"]) + int(r["l3_len"])])
        frames.append(bytes(12) + (b"\x08\x00" if r["l3_ver"] == 4 else b"\x86\xdd") + l3)
    offs, lens, arena = [], [], bytearray()
    for i, f in enumerate(frames):
        arena += bytes(i % 5)
        offs.append(len(arena))
        lens.append(len(f))
        arena += f
    arena = np.frombuffer(bytes(arena) + bytes(64), np.uint8).copy()
    n = len(frames)
    ga, go, gl = dev(arena), dev(np.array(offs, np.uint64)), dev(np.array(lens, np.uint32))
    d1 = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    d2 = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    tu = torch.full((n * V.TUPLE_DTYPE.itemsize,), 0xAB, dtype=torch.uint8, device="cuda")
    V.parse_ether(ga, go, gl, n, d1)
    V.parse_ether(ga, go, gl, n, d2, st, tuples=tu)
    torch.cuda.synchronize()
    assert torch.equal(d1, d2)
    got = tu.cpu().numpy().view(V.TUPLE_DTYPE)
    nacc = 0
    for i, f in enumerate(frames):
        w = O.flow_tuple(f)
        g = got[i]
        assert bytes(g["src"]) == w["src"] and bytes(g["dst"]) == w["dst"], i
        assert bytes(g["sport"]) == w["sport"] and bytes(g["dport"]) == w["dport"], i
        assert (g["l3_ver"], g["l4_proto"], g["tcp_flags"], g["rsv"]) == (w["l3_ver"], w["l4_proto"], w["tcp_flags"], 0), i
        nacc += w["l3_ver"] != 0
    assert nacc > 4000


@pytest.mark.parametrize("service", [False, True])
def test_ctx_parse_frames_tuples(V, orc, service):
    """vpcsum_ctx_parse_frames (PNI parseFrames, GpuCsumBatch.parseFrames): an RX batch in a
    registered arena parsed where it lies, with flow tuples; descriptors, status and tuples equal
    the oracle's, and the descriptors verify the frames through vpcsum_ctx_submit as the
    reference's recompute does.  Two batches back to back exercise both slots.  service: batches
    of up to 400 frames parsed on the service grid (svc_frame_packet, parse only), every byte of
    the results equal to the launched parse kernel's."""
    import edgevec as E
    frames = [f for f, _, _ in E.parse_cases()]
    a, d = orc.synth(600, 2048, 14, O.SYNTH_FUZZ, O.SEED, 99)
    for r in d:
        l3 = bytes(a[int(r["l3_off"]):int(r["l3_off"]) + int(r["l3_len"])])
        frames.append(bytes(12) + (b"\x08\x00" if r["l3_ver"] == 4 else b"\x86\xdd") + l3)
    offs, lens, arena = [], [], bytearray()
    for i, f in enumerate(frames):
        arena += bytes(3 if i % 2 else 0)
        offs.append(len(arena))
        lens.append(len(f))
        arena += f
    arena = np.frombuffer(bytes(arena) + bytes(64), np.uint8).copy()
    n = len(frames)
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
    ctx.register(arena)
    if service:
        ref = ctx.parse_frames(arena, np.array(offs), np.array(lens))   # launched: n > 512
        ctx.set_service(20000)
    for rep in range(2):
        if service:
            parts = [ctx.parse_frames(arena, np.array(offs[lo:lo + 400]), np.array(lens[lo:lo + 400]))
                     for lo in range(0, n, 400)]
            desc, st, tu = (np.concatenate([p_[k] for p_ in parts]) for k in range(3))
            assert desc.tobytes() == ref[0].tobytes() and np.array_equal(st, ref[1]) and tu.tobytes() == ref[2].tobytes()
        else:
            desc, st, tu = ctx.parse_frames(arena, np.array(offs), np.array(lens))
        for i, f in enumerate(frames):
            info, _ = O.parse_ether(f)
            w = O.flow_tuple(f)
            if info is None:
                assert st[i] == O.S_BAD_DESC and tu[i]["l3_ver"] == 0, i
                continue
            assert st[i] == 0
            g = desc[i]
            assert int(g["l3_off"]) == offs[i] + info.l3_off
            assert (g["l3_len"], g["l4_off"], g["l3_ver"], g["l4_proto"], g["flags"]) == \
                (info.l3_len, info.l4_off, info.ver, info.proto, O.desc_flags_for(info))
            assert bytes(tu[i]["src"]) == w["src"] and bytes(tu[i]["dst"]) == w["dst"], i
            assert bytes(tu[i]["sport"]) == w["sport"] and bytes(tu[i]["dport"]) == w["dport"], i
            assert (tu[i]["l4_proto"], tu[i]["tcp_flags"]) == (w["l4_proto"], w["tcp_flags"]), i
    ok = st == 0
    good = np.ascontiguousarray(desc[ok])
    vout, vst = ctx.run(arena, good, O.MODE_VERIFY)
    want, want_st = orc.process(arena, good, O.MODE_VERIFY)
    if service:
        assert ctx.stats()["service_batches"] == 2 * ((n + 399) // 400)
    ctx.close()
    assert np.array_equal(vout, want) and np.array_equal(vst, want_st)


@pytest.mark.parametrize("mode", [0, 0x100, 1, 0x101])   # RFC 1624 / strict Java, wide / byte kernel
def test_nat_ttl_expired_on_gpu(V, orc, mode):
    """TTL / hop limit 0 and 1 under NAT_DEC_TTL (alone, after SET_TTL, with an address rewrite):
    refused with S_BAD_DESC | S_TTL_EXPIRED, nothing written; TTL 2 and 64 decremented.  Both
    entry formats, IPv4 and IPv6, every kernel and mode; statuses and bytes equal the oracle's."""
    rng = np.random.default_rng(77)
    arena, desc = orc.synth(400, 9088, 2, O.SYNTH_FUZZ, O.SEED, 6060)
    rw = np.zeros(len(desc), O.NAT_DTYPE)
    rw.view(np.uint8).reshape(-1, 48)[:, :36] = rng.integers(0, 256, (len(desc), 36), dtype=np.uint8)
    for i, d in enumerate(desc):
        t = int(d["l3_off"]) + (8 if d["l3_ver"] == 4 else 7)
        arena[t] = [0, 1, 2, 64][i % 4]
        rw[i]["mask"] = O.NAT_DEC_TTL | [0, O.NAT_SET_TTL, O.NAT_SRC | O.NAT_DPORT][(i // 4) % 3]
        rw[i]["ttl"] = [0, 1, 2, 9][(i // 12) % 4]
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)
    want = arena.copy()
    want_st = orc.nat_java(want, desc, rw)
    assert (want_st == (O.S_BAD_DESC | O.S_TTL_EXPIRED)).sum() > 100 and (want_st == O.S_DONE).sum() > 100
    got, st = _gpu_nat48(V, arena, desc, rw, mode)
    assert np.array_equal(st, want_st)
    assert np.array_equal(got, want)
    v4 = desc["l3_ver"] == 4
    want4 = arena.copy()
    want4_st = orc.nat4_java(want4, desc[v4], _nat4_of(rw[v4]))
    got4, st4 = _gpu_nat(V, arena, desc[v4], _nat4_of(rw[v4]), mode)
    assert np.array_equal(st4, want4_st) and np.array_equal(got4, want4)


def test_library_restores_callers_device(V, orc):
    """Every context / group entry point runs on its own device and gives the caller's current
    device back (api.cpp DeviceScope): torch's current device is unchanged after create, register,
    submit, wait, service, NAT and destroy.  With two or more GPUs the contexts live on device 1
    while the caller sits on device 0; on a one-GPU box the group is [0, 0] (the save / restore
    path runs, the device cannot differ)."""
    import torch
    ndev = torch.cuda.device_count()
    other = 1 if ndev > 1 else 0
    torch.cuda.set_device(0)
    arena, desc = orc.synth(64, 2048, 14, O.SYNTH_C3, O.SEED, 808)
    want, _ = orc.process(arena, desc)
    g = V.Group([other, 0], max_arena=arena.nbytes, max_pkts=64)
    assert torch.cuda.current_device() == 0
    g.register(arena)
    out, _ = g.run(arena, desc)
    assert np.array_equal(out, want) and torch.cuda.current_device() == 0
    g.unregister(arena)
    out, _ = g.run(arena, desc)
    assert np.array_equal(out, want) and torch.cuda.current_device() == 0
    g.close()
    ctx = V.Context(other, max_arena=arena.nbytes, max_pkts=64)
    ctx.register(arena)
    ctx.set_service(20000)
    out, _ = ctx.run(arena, desc)
    assert np.array_equal(out, want) and torch.cuda.current_device() == 0
    ctx.close()
    assert torch.cuda.current_device() == 0


def test_group_register_unregister_cycle(V, orc):
    """vpcsum_group_unregister_arena: the arena can be registered again afterwards (the page-lock
    was released), batches run zero-copy while registered and staged after; unregistering an arena
    the group does not hold is an error."""
    arena, desc = orc.synth(200, 2048, 14, O.SYNTH_C3, O.SEED, 909)
    want, _ = orc.process(arena, desc)
    g = V.Group([0, 0], max_arena=arena.nbytes, max_pkts=256)
    for _ in range(3):
        g.register(arena)
        out, _ = g.run(arena, desc)
        assert np.array_equal(out, want)
        g.unregister(arena)
    with pytest.raises(V.VpcsumError, match="not registered"):
        g.unregister(arena)
    out, _ = g.run(arena, desc)
    assert np.array_equal(out, want)
    # a zero-copy batch still in flight on the arena: unregister finishes it on every context first
    # (phase 1), then drops the mappings and unpins (phase 2); the results are whole
    g.register(arena)
    out = np.zeros(len(desc), np.uint32)
    t = g.submit(arena, desc, out, None, O.MODE_COMPUTE)
    g.unregister(arena)
    g.wait(t)
    assert np.array_equal(out, want)
    g.register(arena)   # and it registers again
    g.unregister(arena)
    g.close()


def test_default_group_threads_race_shutdown(V, orc):
    """vpcsum_batch_submit / vpcsum_batch_wait from several threads while another thread shuts the
    process-wide group down and re-initialises it: never a use-after-free (the group is
    held under a shared lock for each call, shutdown takes it exclusively), and every submit that
    succeeded gets the oracle's results in its buffer, whether its wait returns 0 or a defined error:
    "vpcsum_init first" (no group) or "before vpcsum_shutdown" (a handle of an earlier group) --
    the shutdown completed the batch."""
    import ctypes
    import threading
    import torch
    L = V.lib()
    mask = 1
    arena, d = orc.synth(512, 2048, 14, O.SYNTH_C3, O.SEED, 2024)
    want, _ = orc.process(arena, d)
    errors, done, after_shutdown = [], [0], [0]
    stop = threading.Event()

    def worker():
        out = np.zeros(len(d), np.uint32)
        h = ctypes.c_uint64()
        while not stop.is_set():
            out[:] = 0
            if L.vpcsum_batch_submit(arena.ctypes.data, arena.nbytes, d.ctypes.data, len(d), out.ctypes.data, None,
                                     0, ctypes.byref(h)) != 0:
                msg = L.vpcsum_last_error().decode()
                if "vpcsum_init first" not in msg:
                    errors.append(msg)
                continue
            if L.vpcsum_batch_wait(h.value) != 0:
                msg = L.vpcsum_last_error().decode()
                if "vpcsum_init first" not in msg and "before vpcsum_shutdown" not in msg:
                    errors.append(msg)
                after_shutdown[0] += 1
            if not np.array_equal(out, want):
                errors.append("a submitted batch's results were not delivered")
            done[0] += 1

    assert L.vpcsum_init(mask, arena.nbytes, len(d)) == 0
    ts = [threading.Thread(target=worker) for _ in range(4)]
    for t in ts:
        t.start()
    try:
        for _ in range(20):
            assert L.vpcsum_shutdown() == 0
            assert L.vpcsum_init(mask, arena.nbytes, len(d)) == 0
    finally:
        stop.set()
        for t in ts:
            t.join(60)
        L.vpcsum_shutdown()
    torch.cuda.synchronize()
    assert not errors, errors[:5]
    assert done[0] > 0


def test_shutdown_completes_batches_and_refuses_old_handles(V, orc):
    """vpcsum_shutdown completes every batch in flight before it frees anything (results in the
    caller's buffers: staged and zero-copy), and a handle from before it is refused after a new
    vpcsum_init instead of naming one of the new group's tickets."""
    import ctypes
    L = V.lib()
    arena, d = orc.synth(700, 2048, 14, O.SYNTH_C3, O.SEED, 4040)
    want, want_st = orc.process(arena, d)
    for reg in (False, True):
        assert L.vpcsum_init(1, arena.nbytes, len(d)) == 0
        try:
            if reg:
                assert L.vpcsum_register_arena(arena.ctypes.data, arena.nbytes) == 0
            outs = [np.zeros(len(d), np.uint32) for _ in range(2)]
            sts = [np.zeros(len(d), np.uint8) for _ in range(2)]
            hs = [ctypes.c_uint64() for _ in range(2)]
            for o, st, h in zip(outs, sts, hs):   # two batches in flight, never waited
                assert L.vpcsum_batch_submit(arena.ctypes.data, arena.nbytes, d.ctypes.data, len(d), o.ctypes.data,
                                             st.ctypes.data, 0, ctypes.byref(h)) == 0
        finally:
            assert L.vpcsum_shutdown() == 0
        for o, st in zip(outs, sts):
            assert np.array_equal(o, want) and np.array_equal(st, want_st), reg
        assert L.vpcsum_init(1, arena.nbytes, len(d)) == 0
        try:
            assert L.vpcsum_batch_wait(hs[1].value) != 0
            assert "before vpcsum_shutdown" in L.vpcsum_last_error().decode()
            h = ctypes.c_uint64()
            out = np.zeros(len(d), np.uint32)
            assert L.vpcsum_batch_submit(arena.ctypes.data, arena.nbytes, d.ctypes.data, len(d), out.ctypes.data,
                                         None, 0, ctypes.byref(h)) == 0
            assert (h.value & ((1 << 48) - 1)) == (hs[0].value & ((1 << 48) - 1))   # the same ticket number ...
            assert h.value != hs[0].value                                            # ... of another generation
            assert L.vpcsum_batch_wait(h.value) == 0 and np.array_equal(out, want)
        finally:
            L.vpcsum_shutdown()


def test_full_size_c5_properties(V, orc):
    """BASELINE config C5 at its full size: 10,000,000 x 1500 B IPv4 TCP/UDP in one 20.5-GB arena,
    every packet's addresses and ports rewritten (RFC 1624, the bench's kernel and mask).
    Every packet is compared with the oracle: the batch is regenerated on the host in 1M-packet
    chunks, checksummed and rewritten by the oracle's Java restatement (setters + full recompute,
    SwitchUtils.java:522-542 -> AbstractPacket.java:58-65), and each chunk's 2-KB frames must equal
    the GPU's byte for byte, whole.  Also, over all 10M packets: every rewritten packet verifies on
    the GPU and the rewritten fields hold the entries' bytes."""
    import torch
    n, stride, chunk = 10_000_000, 2048, 1 << 20
    threads = max(1, min(16, os.cpu_count() or 1))
    arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    V.synth(arena, n, stride, 0, O.SYNTH_C5, O.SEED, 0, d)
    V.compute(arena, d, n, None, None, O.MODE_WRITE)
    g = torch.Generator(device="cpu").manual_seed(55)
    rw = torch.randint(0, 256, (n, 16), dtype=torch.uint8, generator=g)
    rw[:, 12] = O.NAT_SRC | O.NAT_DST | O.NAT_SPORT | O.NAT_DPORT
    rw[:, 13:] = 0
    rw_d = rw.cuda()
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.nat4(arena, d, rw_d, n, st, V.NAT_RFC1624)
    torch.cuda.synchronize()
    assert bool((st == O.S_DONE).all())
    vs = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.compute(arena, d, n, None, vs, O.MODE_VERIFY)
    torch.cuda.synchronize()
    assert bool(((vs & 3) == 3).all()), "a rewritten packet no longer verifies"
    frames = arena.view(n, stride)
    assert torch.equal(frames[:, 12:16].cpu(), rw[:, 0:4]) and torch.equal(frames[:, 16:20].cpu(), rw[:, 4:8])
    assert torch.equal(frames[:, 20:24].cpu(), rw[:, 8:12])      # ports (TCP and UDP: at L4 + 0..3)
    rw_np = rw.numpy().view(O.NAT4_DTYPE).reshape(-1)
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        a, dd = orc.synth(m, stride, 0, O.SYNTH_C5, O.SEED, c0, threads=threads)
        orc.process(a, dd, O.MODE_COMPUTE, write=True, threads=threads)
        orc.nat4_java(a, dd, np.ascontiguousarray(rw_np[c0:c0 + m]), threads=threads)
        got = arena[c0 * stride:(c0 + m) * stride].cpu().numpy()
        if not np.array_equal(got, a):
            bad = np.nonzero((got.reshape(m, stride) != a.reshape(m, stride)).any(axis=1))[0]
            raise AssertionError(f"{len(bad)} packets of [{c0}, {c0 + m}) differ, first {c0 + int(bad[0])}")
        del got, a
    del arena, frames
