"""Window units of K2: when the 64 packets of a unit are small, of one
shape and within 4 KB, the wave reads the unit's window with coalesced loads and each lane sums
its own packet from LDS.  These batches are built so that units take that path, miss it by one
condition (one bad descriptor, one packet of another shape or length, one packet outside the
window, a stride that changes the L3 alignment from packet to packet, a partial unit at the end),
or mix both, and every result is compared with the oracle (compute, verify with corrupted sums,
checksum write-back, CHECKSUM_PARTIAL)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests import edgevec as E
from tests.test_gpu_parity import V, gpu_compute  # noqa: F401  (V: the library fixture)

pytestmark = pytest.mark.gpu

# 0: the default (dense frames take the build without result staging);
# 79: the staging build on the same batches; 72: K2 without window units
VARIANTS = [0, 79, 72]

# (ver, proto, l3_len, flags): shapes whose r0 + l3_len fits the first 64 B of the chunk-aligned
# frame for r0 = 14 (l3_len <= 50) or r0 = 0 (<= 64)
SHAPES_14 = [(4, 17, 50, O.F_IP | O.F_L4), (4, 17, 28, O.F_IP | O.F_L4), (4, 6, 44, O.F_IP | O.F_L4),
             (4, 1, 36, O.F_IP | O.F_L4), (4, 6, 40, O.F_L4), (4, 17, 33, O.F_IP), (6, 17, 50, O.F_L4),
             (6, 58, 47, O.F_L4), (4, 6, 50, O.F_L4P), (6, 17, 48, O.F_L4P), (4, 1, 25, O.F_IP | O.F_L4)]
SHAPES_0 = SHAPES_14 + [(6, 6, 64, O.F_L4), (4, 17, 64, O.F_IP | O.F_L4), (4, 6, 61, O.F_IP | O.F_L4)]


def _packet(rng, ver, proto, l3_len):
    if ver == 4:
        return E._v4(rng, proto, l3_len - 20)
    return E._v6(rng, proto, l3_len - 40)


def build(rng, shapes_of_unit, n, stride, pad, spread=None):
    """n packets at `stride` (packet i at i*stride + pad, or at spread(i) when given); unit u
    (64 packets) takes its shapes from shapes_of_unit(u, i)."""
    at = [spread(i) if spread else i * stride + pad for i in range(n)]
    arena = np.zeros(max(at) + 128, np.uint8)
    rows = []
    for i in range(n):
        ver, proto, l3_len, flags = shapes_of_unit(i // 64, i)
        p, l4 = _packet(rng, ver, proto, l3_len)
        arena[at[i]:at[i] + len(p)] = np.frombuffer(bytes(p), np.uint8)
        rows.append((at[i], l3_len, l4, ver, proto, flags, 0))
    return arena, np.array(rows, dtype=O.DESC_DTYPE)


def check_all(V, orc, arena, desc, variants=VARIANTS):
    """Compute, write-back and verify (after writing the true sums and corrupting a tenth of the
    packets) on each variant; every result equals the oracle's."""
    for v in variants:
        out, st, _ = gpu_compute(V, arena, desc, O.MODE_COMPUTE, v)
        oout, ost = orc.process(arena.copy(), desc, O.MODE_COMPUTE)
        assert np.array_equal(out, oout) and np.array_equal(st, ost), f"variant {v} compute"
        out, st, wr = gpu_compute(V, arena, desc, O.MODE_COMPUTE, v, write=True)
        a2 = arena.copy()
        oout, ost = orc.process(a2, desc, O.MODE_COMPUTE, write=True)
        assert np.array_equal(out, oout) and np.array_equal(wr, a2), f"variant {v} write"
    good = arena.copy()
    orc.process(good, desc, O.MODE_COMPUTE, write=True)
    rng = np.random.default_rng(99)
    for i in np.flatnonzero(rng.random(len(desc)) < 0.1):
        good[int(desc["l3_off"][i]) + int(rng.integers(0, int(desc["l3_len"][i])))] ^= 0x5A
    for v in variants:
        out, st, _ = gpu_compute(V, good, desc, O.MODE_VERIFY, v)
        oout, ost = orc.process(good.copy(), desc, O.MODE_VERIFY)
        assert np.array_equal(out, oout) and np.array_equal(st, ost), f"variant {v} verify"


@pytest.mark.parametrize("shape", range(len(SHAPES_14)))
def test_uniform_units_r14(V, orc, shape):
    """Every unit one shape, 64-B frames, L3 at 14: all units but the partial last one take the
    window path."""
    rng = np.random.default_rng(shape)
    arena, desc = build(rng, lambda u, i: SHAPES_14[shape], 64 * 9 + 17, 64, 14)
    check_all(V, orc, arena, desc)


@pytest.mark.parametrize("shape", range(len(SHAPES_0)))
def test_uniform_units_r0(V, orc, shape):
    rng = np.random.default_rng(100 + shape)
    arena, desc = build(rng, lambda u, i: SHAPES_0[shape], 64 * 5, 64, 0)
    check_all(V, orc, arena, desc)


@pytest.mark.parametrize("stride,pad", [(48, 2), (32, 0), (80, 14), (64, 30), (128, 14), (52, 14), (64, 15)])
def test_strides(V, orc, stride, pad):
    """Denser and sparser strides (a 4-KB window holds fewer than 64 frames at 80 and 128 B), a
    stride that moves the alignment from packet to packet (52), an odd L3 start (15)."""
    rng = np.random.default_rng(stride + pad)
    fit = min(stride, 64) - (pad & 15) if stride >= 32 else 28
    shapes = [s for s in SHAPES_0 if s[2] <= fit and (s[0] == 4 and s[2] >= 28 or s[2] >= 48)]
    arena, desc = build(rng, lambda u, i: shapes[u % len(shapes)], 64 * 7, stride, pad)
    check_all(V, orc, arena, desc)


def test_units_that_miss_by_one(V, orc):
    """Unit 0 uniform; unit 1 one packet of another length; unit 2 one of another protocol; unit 3
    one bad descriptor; unit 4 one packet far outside the window; unit 5 packets in reverse order
    (lane 0 holds the highest offset); unit 6 uniform again."""
    rng = np.random.default_rng(7)
    n = 64 * 7
    base_shape = (4, 17, 50, O.F_IP | O.F_L4)

    def shapes(u, i):
        if u == 1 and i % 64 == 13:
            return (4, 17, 44, O.F_IP | O.F_L4)
        if u == 2 and i % 64 == 40:
            return (4, 6, 50, O.F_IP | O.F_L4)
        return base_shape

    def spread(i):
        u, k = divmod(i, 64)
        if u == 4 and k == 63:
            return 64 * n + 14
        if u == 5:
            return (u * 64 + 63 - k) * 64 + 14
        return i * 64 + 14

    arena, desc = build(rng, shapes, n, 64, 14, spread)
    desc["l3_ver"][3 * 64 + 5] = 5
    check_all(V, orc, arena, desc)


def test_c1_synth_window(V, orc):
    """The C1 generator at its bench stride (64-B frames, L3 at 14), 3000 packets."""
    arena, desc = orc.synth(3000, 64, 14, O.SYNTH_C1, O.SEED, 555)
    check_all(V, orc, arena, desc)


@pytest.mark.parametrize("registered", [False, True])
def test_window_units_host_context(V, orc, registered):
    """Dense small frames from host memory: staged through the context's device buffers
    (pageable arena) or read in place from a registered one (zero-copy), verify then write-back;
    batches large enough that K2 (not the one-wave-per-packet zero-copy variant) runs."""
    rng = np.random.default_rng(31)
    arena, desc = build(rng, lambda u, i: SHAPES_14[u % 4], 64 * 40 + 5, 64, 14)
    good = arena.copy()
    orc.process(good, desc, O.MODE_COMPUTE, write=True)
    for i in range(0, len(desc), 7):
        good[int(desc["l3_off"][i]) + 20] ^= 0x11
    ctx = V.Context(0, max_arena=good.nbytes, max_pkts=len(desc))
    try:
        if registered:
            ctx.register(good)
        out, st = ctx.run(good, desc, O.MODE_VERIFY)
        oout, ost = orc.process(good.copy(), desc, O.MODE_VERIFY)
        assert np.array_equal(out, oout) and np.array_equal(st, ost)
        want = good.copy()
        wout, _ = orc.process(want, desc, O.MODE_COMPUTE, write=True)
        out = np.zeros(len(desc), np.uint32)
        ctx.wait(ctx.submit(good, desc, out, None, O.MODE_WRITE))
        assert np.array_equal(out, wout) and np.array_equal(good, want)
    finally:
        ctx.close()


@pytest.mark.parametrize("stride,pad", [(2048, 14), (2048, 0), (4096, 2), (192, 14)])
def test_gathered_units(V, orc, stride, pad):
    """Small packets of one shape in sparse frames (2-KB umem frames and others): not within one
    4-KB window, so the unit's chunks are gathered per packet; shapes of 1 to 4 chunks."""
    rng = np.random.default_rng(stride + pad)
    fit = 64 - (pad & 15)
    shapes = [s for s in SHAPES_0 if s[2] <= fit]
    arena, desc = build(rng, lambda u, i: shapes[u % len(shapes)], 64 * len(shapes) + 9, stride, pad)
    check_all(V, orc, arena, desc)


def test_gathered_units_shuffled(V, orc):
    """Descriptors in random order over 64-B frames (not ascending, so not a window), and units
    whose frames lie in reverse order."""
    rng = np.random.default_rng(5)
    arena, desc = build(rng, lambda u, i: SHAPES_14[0], 64 * 12, 64, 14)
    perm = rng.permutation(len(desc))
    check_all(V, orc, arena, desc[perm].copy())
    check_all(V, orc, arena, desc[::-1].copy())


def test_c1_synth_umem_frames(V, orc):
    """The C1 generator in 2-KB frames (the AF_XDP umem layout), 3000 packets."""
    arena, desc = orc.synth(3000, 2048, 14, O.SYNTH_C1, O.SEED, 77)
    check_all(V, orc, arena, desc)
