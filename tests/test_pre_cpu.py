"""The pre-image flush on the CPU (no GPU): the seam's host logic and the arithmetic it relies on.

* `vswitch.record_pre_image` records exactly the words Java's setters then overwrite
  (SwitchUtils.applyNat -> setSrc / setDst / setSrcPort / setDstPort, SwitchUtils.java:531-542),
  checked against the oracle's setters (oracle/csum_oracle.c:orc_nat_apply).
* RFC 1624 eqn. 3 from those pre-images, restated here in Python as the kernels apply it
  (nat.hip / pre_common.h:pre_sums; the service grid's svc_pre_packet), equals Java's full
  recompute (getRawPacket(0), AbstractPacket.java:58-65 -> oracle) on every packet whose stored L4
  sum was correct, and differs where it was not -- the reason `vswitch.pre_eligible` gates F_PRE
  on ingress verify's S_L4_OK.
The GPU tests (tests/test_gpu_pre.py) then hold the kernels to the same oracle.
"""
import numpy as np

from oracle import oracle as O

NAT_FIELDS = O.NAT_SRC | O.NAT_DST | O.NAT_SPORT | O.NAT_DPORT


def _ld16(a, o):
    return (int(a[o]) << 8) | int(a[o + 1])


def _fold(x):
    while x >> 16:
        x = (x & 0xFFFF) + (x >> 16)
    return x


def _words(b):
    return [(int(b[i]) << 8) | int(b[i + 1]) for i in range(0, len(b), 2)]


def rfc1624_from_pre(frame, d, pre):
    """The L4 sum the flush writes for F_PRE packet d (frame after the setters), or None when the
    frame's stored sum is a UDP 0 (the kernels then sum the segment in full, as Java does)."""
    l3, ver, proto, l4o = int(d["l3_off"]), int(d["l3_ver"]), int(d["l4_proto"]), int(d["l4_off"])
    hc = _ld16(frame, l3 + l4o + O.L4_FIELD[proto])
    if proto == 17 and hc == 0:
        return None
    ports = proto in (6, 17)
    addr = ports or (ver == 6 and proto == 58)
    alen, a0 = (4, 12) if ver == 4 else (16, 8)
    diff = 0
    if addr:
        for bit, name, off in ((O.NAT_SRC, "src", a0), (O.NAT_DST, "dst", a0 + alen)):
            if pre["mask"] & bit:
                for m, m2 in zip(_words(pre[name][:alen]), _words(frame[l3 + off:l3 + off + alen])):
                    diff += (~m & 0xFFFF) + m2
    if ports:
        for bit, name, off in ((O.NAT_SPORT, "sport", 0), (O.NAT_DPORT, "dport", 2)):
            if pre["mask"] & bit:
                diff += (~_words(pre[name])[0] & 0xFFFF) + _ld16(frame, l3 + l4o + off)
    c = ~_fold((~hc & 0xFFFF) + _fold(diff)) & 0xFFFF
    return 0xFFFF if proto == 17 and c == 0 else c


def _case(orc, seed, n, workload, stride=9088):
    from vproxy_amd import vswitch as S
    rng = np.random.default_rng(seed)
    arena, desc = orc.synth(n, stride, 14, workload, O.SEED, seed)
    orc.process(arena, desc, O.MODE_COMPUTE, write=True)
    for d in desc:                                     # some UDP "no checksum" packets
        if d["l4_proto"] == 17 and rng.random() < 0.1:
            o = int(d["l3_off"]) + int(d["l4_off"])
            arena[o + 6:o + 8] = 0
    rw = np.zeros(n, O.NAT_DTYPE)
    rw.view(np.uint8).reshape(n, 48)[:, :36] = rng.integers(0, 256, (n, 36), dtype=np.uint8)
    rw["mask"] = rng.integers(1, 16, n)
    pre = np.zeros(n, O.NAT_DTYPE)
    for i, d in enumerate(desc):
        pre[i] = S.record_pre_image(arena, int(d["l3_off"]), int(d["l3_ver"]), int(d["l4_off"]), int(d["l4_proto"]),
                                    int(rw[i]["mask"]))
    return rng, arena, desc, rw, pre


def test_pre_image_holds_the_words_the_setters_overwrite(orc):
    """Every byte the oracle's setters change lies in a field the pre-image recorded, and the
    pre-image holds its old value; fields outside the mask are left zero, ports only for TCP / UDP."""
    _, arena, desc, rw, pre = _case(orc, 3, 600, O.SYNTH_FUZZ)
    after = arena.copy()
    orc.nat_setters(after, desc, rw)
    for i, d in enumerate(desc):
        l3, ver, proto, l4o = int(d["l3_off"]), int(d["l3_ver"]), int(d["l4_proto"]), int(d["l4_off"])
        alen, a0 = (4, 12) if ver == 4 else (16, 8)
        fields = [("src", l3 + a0, alen, O.NAT_SRC), ("dst", l3 + a0 + alen, alen, O.NAT_DST)]
        if proto in (6, 17):
            fields += [("sport", l3 + l4o, 2, O.NAT_SPORT), ("dport", l3 + l4o + 2, 2, O.NAT_DPORT)]
        covered = np.zeros(len(arena), bool)
        for name, off, ln, bit in fields:
            if rw[i]["mask"] & bit:
                assert pre[i]["mask"] & bit, i
                assert bytes(pre[i][name][:ln]) == bytes(arena[off:off + ln]), (i, name)
                covered[off:off + ln] = True
            else:
                assert not pre[i]["mask"] & bit and not pre[i][name].any(), (i, name)
        if proto not in (6, 17):
            assert not pre[i]["mask"] & (O.NAT_SPORT | O.NAT_DPORT) and not pre[i]["sport"].any()
        seg = slice(l3, l3 + int(d["l3_len"]))
        changed = np.nonzero(after[seg] != arena[seg])[0] + l3
        assert covered[changed].all(), i


def test_rfc1624_from_pre_images_equals_java_on_valid_sums(orc):
    """On frames whose stored L4 sums were correct, eqn. 3 from the pre-image and the words now in
    the frame gives Java's full recompute, for IPv4 and IPv6, TCP / UDP / ICMP / ICMPv6, every mask,
    sums of 0 (UDP 0 -> 0xffff); UDP stored 0 is summed in full (None here) and stays Java's."""
    checked = 0
    for seed, workload in ((4, O.SYNTH_FUZZ), (5, O.SYNTH_C5), (6, O.SYNTH_C3)):
        _, arena, desc, rw, pre = _case(orc, seed, 800, workload)
        want = arena.copy()
        st = orc.nat_java(want, desc, rw)
        after = arena.copy()
        orc.nat_setters(after, desc, rw)
        for i, d in enumerate(desc):
            proto, ver = int(d["l4_proto"]), int(d["l3_ver"])
            if st[i] != O.S_DONE or proto not in O.L4_FIELD or (ver == 4 and proto == 58):
                continue
            l3, l4o = int(d["l3_off"]), int(d["l4_off"])
            f = l3 + l4o + O.L4_FIELD[proto]
            if int(d["l3_len"]) - l4o < O.L4_FIELD[proto] + 2:
                continue
            c = rfc1624_from_pre(after, d, pre[i])
            if c is None:   # UDP stored 0: summed in full by the kernels, as by Java
                assert proto == 17 and _ld16(after, f) == 0, i
                continue
            assert c == _ld16(want, f), (i, ver, proto, hex(c), hex(_ld16(want, f)))
            checked += 1
    assert checked > 1500


def test_rfc1624_from_pre_images_diverges_on_invalid_sums(orc):
    """A payload byte changed after the stored sum was taken (what ingress verify reports as not
    S_L4_OK): the incremental update carries the error along, Java's recompute does not -- those
    frames must take the full path."""
    from vproxy_amd import vswitch as S
    _, arena, desc, rw, pre = _case(orc, 7, 400, O.SYNTH_C5, stride=2048)
    rw["mask"] = NAT_FIELDS
    for i, d in enumerate(desc):
        arena[int(d["l3_off"]) + 700] ^= 0x5A        # invalidates the stored L4 sum
        pre[i] = S.record_pre_image(arena, int(d["l3_off"]), 4, int(d["l4_off"]), int(d["l4_proto"]), NAT_FIELDS)
    want = arena.copy()
    orc.nat_java(want, desc, rw)
    after = arena.copy()
    orc.nat_setters(after, desc, rw)
    differ = compared = 0
    for i, d in enumerate(desc):
        f = int(d["l3_off"]) + int(d["l4_off"]) + O.L4_FIELD[int(d["l4_proto"])]
        c = rfc1624_from_pre(after, d, pre[i])
        if c is not None:
            compared += 1
            differ += c != _ld16(want, f)
    assert compared > 300 and differ >= 0.99 * compared


def test_pre_eligible_follows_ingress_verify():
    """F_PRE only for a frame whose stored L4 sum ingress verify proved (S_L4_OK), never for a
    refused frame or one verified without it (corrupt, CHECKSUM_PARTIAL, UDP stored 0)."""
    from vproxy_amd import vswitch as S
    assert S.pre_eligible(O.S_DONE | O.S_IP_OK | O.S_L4_OK)
    assert S.pre_eligible(O.S_DONE | O.S_L4_OK)
    assert not S.pre_eligible(O.S_DONE | O.S_IP_OK)
    assert not S.pre_eligible(O.S_DONE | O.S_IP_OK | O.S_UDP_NOCSUM)
    assert not S.pre_eligible(O.S_BAD_DESC | O.S_L4_OK)
    assert not S.pre_eligible(0)
