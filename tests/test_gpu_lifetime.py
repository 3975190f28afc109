"""Host-memory lifetimes around registration (VERDICT r5 "Next round" item 2).

The sequence round 5's two intermittent faults fit (DESIGN_HISTORY.md "Round 6: the intermittent
fault"): a range page-locked for zero-copy batches is released -- unregistered, or its context /
group / the process-wide group destroyed -- the memory is freed, the allocator hands the same
addresses to a new array, and torch copies that new array to the device with an ordinary
PAGEABLE host-to-device copy, whose result a kernel then reads.  If HIP still held the old range as
registered, the copy would go through the dead registration's mapping.

Each test runs that sequence deterministically, many times, on every release path of the library,
with pageable copies (no pin_memory), and checks at each step what HIP believes
(vpcsum.hip_holds_registered) before the copy, and the kernel's results after it.  The staged submit
is checked not to copy straight from memory the context did not register (is_registered).
"""
import ctypes

import numpy as np
import pytest

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


def _pageable_roundtrip(V, orc, n, seed):
    """A fresh numpy batch -> torch's pageable H2D copy -> the checksum kernel -> the oracle's
    sums.  Returns the arena's address (to see whether the allocator reused the released one)."""
    import torch
    arena, desc = orc.synth(n, 2048, 14, O.SYNTH_C3, O.SEED, seed)
    assert not V.hip_holds_registered(arena.ctypes.data), "a fresh array is held as registered"
    a = torch.from_numpy(arena).cuda()                  # pageable: no pin_memory
    d = torch.from_numpy(desc.view(np.uint8).reshape(-1)).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    V.compute(a, d, n, out)
    torch.cuda.synchronize()
    want, _ = orc.process(arena, desc)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    return arena.ctypes.data


def _zero_copy_batch(V, orc, runner, arena, desc):
    want, _ = orc.process(arena, desc)
    out, _ = runner.run(arena, desc)
    assert np.array_equal(out, want)


@pytest.mark.parametrize("release", ["unregister", "ctx_close", "group_unregister", "group_close"])
def test_release_free_reallocate_pageable_copy(V, orc, release):
    """register -> zero-copy batch -> release -> the range is no longer registered -> free ->
    reallocate the same size -> pageable H2D -> kernel: 25 rounds, sizes 200..2000 packets (the
    allocator reuses the released addresses in most rounds: counted, and required at least once)."""
    reused = 0
    for r in range(25):
        n = 200 + 75 * r
        arena, desc = orc.synth(n, 2048, 14, O.SYNTH_C3, O.SEED, 1000 + r)
        ptr, nbytes = arena.ctypes.data, arena.nbytes
        if release.startswith("group"):
            h = V.Group((0, 0), max_arena=nbytes, max_pkts=n)
        else:
            h = V.Context(0, max_arena=nbytes, max_pkts=n)
        h.register(arena)
        assert V.hip_holds_registered(ptr)
        _zero_copy_batch(V, orc, h, arena, desc)
        if release.endswith("unregister"):
            h.unregister(arena)
            assert not V.hip_holds_registered(ptr) and not V.hip_holds_registered(ptr + nbytes - 1)
            h.close()
        else:
            h.close()
            assert not V.hip_holds_registered(ptr) and not V.hip_holds_registered(ptr + nbytes - 1)
        del arena, desc, h
        reused += _pageable_roundtrip(V, orc, n, 2000 + r) == ptr
    assert reused >= 1


def test_default_group_shutdown_then_pageable_copy(V, orc):
    """The process-wide group (vpcsum_init / vpcsum_register_arena / vpcsum_shutdown): after the
    shutdown the arena is no longer registered, and a pageable copy of a new array at its
    addresses feeds the kernel correctly."""
    L = V.lib()
    for r in range(10):
        n = 300 + 100 * r
        arena, desc = orc.synth(n, 2048, 14, O.SYNTH_C3, O.SEED, 3000 + r)
        ptr, nbytes = arena.ctypes.data, arena.nbytes
        assert L.vpcsum_init(1, nbytes, n) == 0
        try:
            assert L.vpcsum_register_arena(ctypes.c_void_p(ptr), ctypes.c_uint64(nbytes)) == 0
            out = np.zeros(n, np.uint32)
            h = ctypes.c_uint64()
            assert L.vpcsum_batch_submit(arena.ctypes.data, nbytes, desc.ctypes.data, n, out.ctypes.data, None, 0,
                                         ctypes.byref(h)) == 0
            assert L.vpcsum_batch_wait(h.value) == 0
            assert np.array_equal(out, orc.process(arena, desc)[0])
        finally:
            assert L.vpcsum_shutdown() == 0
        assert not V.hip_holds_registered(ptr) and not V.hip_holds_registered(ptr + nbytes - 1)
        del arena, desc
        _pageable_roundtrip(V, orc, n, 4000 + r)


def test_staged_submit_does_not_copy_from_memory_it_did_not_register(V, orc):
    """A staged submit (the context did not register the arena) from an arena another context has
    page-locked: the batch is copied through the context's own staging, so the other context may
    unregister it -- and the memory be freed -- right after the submit, with the batch still in
    flight, and the results are whole."""
    for r in range(8):
        n = 1500
        arena, desc = orc.synth(n, 2048, 14, O.SYNTH_C3, O.SEED, 5000 + r)
        want, _ = orc.process(arena, desc)
        owner = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
        owner.register(arena)
        user = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
        out = np.zeros(n, np.uint32)
        t = user.submit(arena, desc, out)
        owner.unregister(arena)
        owner.close()
        arena[:] = 0          # the caller reuses its buffer: the staged copy was taken at submit
        user.wait(t)
        assert np.array_equal(out, want), r
        user.close()


def test_one_range_registered_by_two_contexts(V, orc):
    """HIP keys a host registration by its start address (profiles/r06c_reg_probe.jsonl): a second
    hipHostRegister of a registered start returns success without a registration of its own, the
    first hipHostUnregister drops it for both holders and the second fails -- so round 5's library
    left the second context with a dead mapping.  Now both contexts hold references on one
    page-lock: either may unregister first, the other's zero-copy batches still run, and the range
    is unpinned with the last reference; a sub-range shares the lock too."""
    n = 500
    arena, desc = orc.synth(n, 2048, 14, O.SYNTH_C3, O.SEED, 6000)
    for first in ("a", "b"):
        a = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
        b = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
        a.register(arena)
        b.register(arena)                                  # shared, not a second hipHostRegister
        sub = arena[2048 * 100:]                           # a sub-range: shares the lock as well
        c = V.Context(0, max_arena=sub.nbytes, max_pkts=n)
        c.register(sub)
        x, y = (a, b) if first == "a" else (b, a)
        x.unregister(arena)
        assert V.hip_holds_registered(arena.ctypes.data)  # still pinned: y holds a reference
        _zero_copy_batch(V, orc, y, arena, desc)
        d2 = desc[200:].copy()
        d2["l3_off"] -= 2048 * 100
        _zero_copy_batch(V, orc, c, sub, d2)
        c.close()
        y.close()
        assert not V.hip_holds_registered(arena.ctypes.data)
        x.close()
    del arena
    _pageable_roundtrip(V, orc, n, 6001)


def test_overlapping_and_foreign_ranges_are_refused(V, orc):
    """A range that partially overlaps a page-locked arena, and memory HIP already holds as
    page-locked by another owner (a torch pinned tensor), are refused: registering them would be a
    second registration HIP does not keep (the lock's lifetime belongs to its owner).  A staged
    submit from such memory still works (copied through the context's staging)."""
    import torch
    n = 300
    arena, desc = orc.synth(n, 2048, 14, O.SYNTH_C3, O.SEED, 6100)
    a = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
    b = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
    a.register(arena[: 2048 * 200])
    with pytest.raises(V.VpcsumError, match="overlaps"):
        b.register(arena[2048 * 100:])
    a.close()
    b.register(arena[2048 * 100:])                         # fine once the first lock is gone
    b.close()
    pinned = torch.from_numpy(arena).pin_memory()
    pa = pinned.numpy()
    assert V.hip_holds_registered(pa.ctypes.data)
    with pytest.raises(V.VpcsumError, match="outside libvpcsum"):
        b2 = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
        try:
            b2.register(pa)
        finally:
            b2.close()
    c = V.Context(0, max_arena=arena.nbytes, max_pkts=n)
    out, _ = c.run(pa, desc)
    assert np.array_equal(out, orc.process(arena, desc)[0])
    c.close()
