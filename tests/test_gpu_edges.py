"""GPU parity on crafted edge vectors (tests/edgevec.py): every rule the reference applies at an
edge is asserted by value on every kernel path, not reached by chance.

* L4 results of 0: UDP stores 0xffff (UdpPacket.java:142-144, 157-159), TCP / ICMP / ICMPv6 keep
  0x0000; IPv4 header results of 0x0000.
* ICMPv4 inside IPv6 (no pseudo header, Ipv6Packet.java:232-234).
* IPv6 with one extension header (odd and even l4_off) through compute, verify, write and the
  pseudo-only offload sum (F_L4P).
* UDP with stored 0 (UDP_NOCSUM).
* NAT (RFC 1624 and strict Java) on UDP whose stored sum is the substituted 0xffff, and rewrites
  whose new sum is 0 (UDP -> 0xffff, TCP 0x0000).

Paths: K2 (default; fast class at even alignment, slow class at odd alignment / odd l4_off),
k_csum team variants, variant 12 (one wave per packet, predicated loads), the host context
(staging copy, zero-copy registered arena, the persistent service grid) and the NAT kernels.
"""
import numpy as np
import pytest

import edgevec as E
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def V():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vproxy_amd import vpcsum
    vpcsum.lib()
    return vpcsum


@pytest.fixture(scope="module")
def packets():
    pk = E.edge_packets(np.random.default_rng(2024))
    E.check_pins(pk)
    return pk


def _gpu(V, arena_np, desc_np, mode, team=0):
    import torch
    arena = torch.from_numpy(arena_np.copy()).pin_memory().cuda()
    n = len(desc_np)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    V.compute(arena, V.desc_to_tensor(desc_np), n, out, st, mode, team)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32), st.cpu().numpy(), arena.cpu().numpy()


def _zero_fields(arena, desc):
    a = arena.copy()
    for d in desc:
        o = int(d["l3_off"])
        if d["l3_ver"] == 4:
            a[o + 10:o + 12] = 0
        f = o + int(d["l4_off"]) + O.L4_FIELD[int(d["l4_proto"])]
        a[f:f + 2] = 0
    return a


def _assert_pins(packets, out):
    for p, o in zip(packets, out):
        if p["want_l4"] is not None:
            assert int(o) >> 16 == p["want_l4"], p["kind"]
        if p["want_ip"] is not None:
            assert int(o) & 0xFFFF == p["want_ip"], p["kind"]


TEAMS = [0, 2, 3, 6, 9, 12, 40, 45, 46, 47, 50, 62, 66, 70, 74]


@pytest.mark.parametrize("pad", [0, 1, 14])
@pytest.mark.parametrize("team", TEAMS)
def test_edges_verify_and_write(V, orc, packets, pad, team):
    arena, desc = E.pack(packets, pad)
    # verify on valid frames: every sum matches, UDP 0xffff is L4_OK, stored 0 is UDP_NOCSUM
    out, st, _ = _gpu(V, arena, desc, O.MODE_VERIFY, team)
    oout, ost = orc.process(arena, desc, O.MODE_VERIFY)
    assert np.array_equal(out, oout) and np.array_equal(st, ost)
    _assert_pins(packets, out)
    nocsum = np.array([p["kind"] == "udp_nocsum" for p in packets])
    assert np.all(st[~nocsum] & O.S_L4_OK) and not np.any(st[nocsum] & O.S_L4_OK)
    assert np.all(st[nocsum] & O.S_UDP_NOCSUM) and not np.any(st[~nocsum] & O.S_UDP_NOCSUM)
    v4 = desc["l3_ver"] == 4
    assert np.all(st[v4] & O.S_IP_OK)
    # write from zeroed fields: the frames come back as the reference writes them
    z = _zero_fields(arena, desc)
    out, st, after = _gpu(V, z, desc, O.MODE_WRITE, team)
    want = z.copy()
    oout, ost = orc.process(want, desc, O.MODE_COMPUTE, write=True)
    assert np.array_equal(out, oout) and np.array_equal(st, ost)
    assert np.array_equal(after, want)
    # ... and equal the valid input frames, except the UDP field of the stored-0 packets
    diff = set(np.nonzero(after != arena)[0].tolist())
    allowed = set()
    for p, d in zip(packets, desc):
        if p["kind"] == "udp_nocsum":
            f = int(d["l3_off"]) + int(d["l4_off"]) + 6
            allowed |= {f, f + 1}
    assert diff <= allowed
    _assert_pins(packets, out)


@pytest.mark.parametrize("pad", [0, 1, 14])
@pytest.mark.parametrize("team", [0, 2, 12, 40, 46, 62])
def test_edges_pseudo_partial(V, orc, packets, pad, team):
    """F_L4P (VP_CSUM_UP_PSEUDO) on the edge packets: ICMPv4 (also inside IPv6) is rejected, the
    rest -- IPv6 extension headers included -- gets the folded pseudo-header sum."""
    arena, desc = E.pack(packets, pad)
    desc = desc.copy()
    desc["flags"] = np.where(desc["l3_ver"] == 4, O.F_IP, 0) | O.F_L4P
    for mode, write in ((O.MODE_COMPUTE, False), (O.MODE_VERIFY, False), (O.MODE_COMPUTE, True)):
        out, st, after = _gpu(V, arena, desc, mode | (O.MODE_WRITE if write else 0), team)
        want = arena.copy()
        oout, ost = orc.process(want, desc, mode, write=write)
        assert np.array_equal(out, oout) and np.array_equal(st, ost), (mode, write)
        assert np.array_equal(after, want)
        icmp4 = desc["l4_proto"] == 1
        assert np.all(st[icmp4] == O.S_BAD_DESC) and not np.any(st[~icmp4] & O.S_BAD_DESC)
        # pure-Python restatement of the pseudo-header sum
        for p, d, o in zip(packets, desc, out):
            if p["proto"] != 1:
                info = O.L3Info(0, p["l3_len"], p["l4_off"], p["ver"], p["proto"])
                assert int(o) >> 16 == O.pseudo_partial(p["bytes"], info), p["kind"]


@pytest.mark.parametrize("service", [0, 20000])
def test_edges_host_context(V, orc, packets, service):
    """The same vectors through the host context: staging copy (pageable arena), zero-copy on a
    registered arena (one wave per packet), and the service grid for small flushes."""
    arena, desc = E.pack(packets, 14)
    arena = np.concatenate([arena, np.zeros(4096, np.uint8)])
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=len(desc))
    try:
        if not service:
            out, st = ctx.run(arena, desc, O.MODE_VERIFY)    # pageable: staged
            oout, ost = orc.process(arena, desc, O.MODE_VERIFY)
            assert np.array_equal(out, oout) and np.array_equal(st, ost)
        ctx.register(arena)
        if service:
            ctx.set_service(service)
        for lo in range(0, len(desc), 37 if service else len(desc)):
            dsc = desc[lo:lo + (37 if service else len(desc))].copy()
            out, st = ctx.run(arena, dsc, O.MODE_VERIFY)
            oout, ost = orc.process(arena, dsc, O.MODE_VERIFY)
            assert np.array_equal(out, oout) and np.array_equal(st, ost), lo
            _assert_pins(packets[lo:lo + len(dsc)], out)
        z = _zero_fields(arena, desc)
        arena[:] = z
        for lo in range(0, len(desc), 3 if service else len(desc)):    # 3: inline descriptors
            dsc = desc[lo:lo + (3 if service else len(desc))].copy()
            want = arena.copy()
            oout, _ = orc.process(want, dsc, O.MODE_COMPUTE, write=True)
            out = np.zeros(len(dsc), np.uint32)
            ctx.wait(ctx.submit(arena, dsc, out, None, O.MODE_WRITE))
            assert np.array_equal(out, oout) and np.array_equal(arena, want), lo
        if service:
            assert ctx.stats()["service_batches"] > 0
    finally:
        ctx.close()


@pytest.mark.parametrize("service", [False, True])
def test_edges_parsed_and_verified(V, orc, packets, service):
    """Received frames (Ethernet + the edge packets) parsed and verified on the GPU in one
    submission: ICMPv4-in-IPv6 and extension-header frames get the reference's verdicts."""
    frames = E.ether_frames(packets)
    offs, lens, arena = [], [], bytearray()
    rng = np.random.default_rng(5)
    for f in frames:
        arena += bytes(int(rng.integers(0, 16)))
        offs.append(len(arena))
        lens.append(len(f))
        arena += f
    arena = np.frombuffer(bytes(arena) + bytes(4096), np.uint8).copy()
    ctx = V.Context(0, max_arena=arena.nbytes, max_pkts=len(frames))
    ctx.register(arena)
    if service:
        ctx.set_service(20000)
    out, st = ctx.verify_frames(arena, np.array(offs), np.array(lens))
    assert ctx.stats()["service_batches"] == (1 if service and len(frames) <= 512 else 0)
    ctx.close()
    for i, f in enumerate(frames):
        info, err = O.parse_ether(f)
        assert info is not None, err
        one = np.array([(offs[i] + info.l3_off, info.l3_len, info.l4_off, info.ver, info.proto,
                         O.desc_flags_for(info), 0)], dtype=O.DESC_DTYPE)
        o, s = orc.process(arena, one, O.MODE_VERIFY)
        assert st[i] == s[0] and out[i] == o[0], (i, packets[i]["kind"])
    _assert_pins(packets, out)


# ---- NAT on the edges ----

def _nat_rw(rng, n):
    rw = np.zeros(n, O.NAT4_DTYPE)
    rw["src"] = rng.integers(0, 256, (n, 4))
    rw["dst"] = rng.integers(0, 256, (n, 4))
    rw["sport"] = rng.integers(0, 256, (n, 2))
    rw["dport"] = rng.integers(0, 256, (n, 2))
    rw["mask"] = O.NAT_SRC | O.NAT_DST | O.NAT_SPORT | O.NAT_DPORT
    return rw


def _force_nat_zero(arena, d, r):
    """Choose the new destination port so that Java's recompute after the rewrite gives an L4
    result of 0 (UDP then stores 0xffff)."""
    o, l4o, proto = int(d["l3_off"]), int(d["l4_off"]), int(d["l4_proto"])
    pkt = bytearray(arena[o:o + int(d["l3_len"])].tobytes())
    pkt[12:16] = bytes(r["src"])
    pkt[16:20] = bytes(r["dst"])
    pkt[l4o:l4o + 2] = bytes(r["sport"])
    pkt[l4o + 2:l4o + 4] = b"\x00\x00"
    c = E.l4_value(bytes(pkt), len(pkt), l4o, 4, proto)
    if proto == 17 and c == 0xFFFF:
        c = 0
    r["dport"] = [c >> 8, c & 0xFF]


def _gpu_nat(V, arena_np, desc, rw, mode):
    import torch
    arena = torch.from_numpy(arena_np.copy()).pin_memory().cuda()
    st = torch.zeros(len(desc), dtype=torch.uint8, device="cuda")
    V.nat4(arena, V.desc_to_tensor(desc), torch.from_numpy(rw.view(np.uint8).copy()).pin_memory().cuda(), len(desc), st, mode)
    torch.cuda.synchronize()
    return arena.cpu().numpy(), st.cpu().numpy()


@pytest.mark.parametrize("pad", [0, 1, 14])
def test_nat_edges(V, orc, packets, pad):
    """IPv4 TCP / UDP edge packets (stored UDP 0xffff among them) rewritten by RFC 1624 and by
    strict Java; half of the rewrites are chosen so that the new sum is 0."""
    sel = [p for p in packets if p["ver"] == 4 and p["proto"] in (6, 17) and p["kind"] != "udp_nocsum"]
    arena, desc = E.pack(sel, pad)
    rng = np.random.default_rng(pad + 3)
    rw = _nat_rw(rng, len(desc))
    for i in range(0, len(desc), 2):
        _force_nat_zero(arena, desc[i], rw[i])
    want = arena.copy()
    orc.nat4_java(want, desc, rw)
    stored_ffff = sum(int.from_bytes(arena[int(d["l3_off"]) + int(d["l4_off"]) + 6:][:2].tobytes(), "big") == 0xFFFF
                      for d in desc if d["l4_proto"] == 17)
    assert stored_ffff > 5
    forced = [int.from_bytes(want[int(d["l3_off"]) + int(d["l4_off"]) + O.L4_FIELD[int(d["l4_proto"])]:][:2].tobytes(), "big")
              for d in desc[::2]]
    assert set(forced) <= {0, 0xFFFF} and 0 in forced and 0xFFFF in forced
    # 0x800000: the lane-layout wide kernel (k_natw) instead of the default quads (k_natq)
    for mode in (0, 0x100, 0x800000, V.NAT_STRICT_JAVA, V.NAT_STRICT_JAVA | 0x100, V.NAT_STRICT_JAVA | 0x800000):
        got, st = _gpu_nat(V, arena, desc, rw, mode)
        assert np.array_equal(got, want), hex(mode)
