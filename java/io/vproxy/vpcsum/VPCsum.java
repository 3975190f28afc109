package io.vproxy.vpcsum;

import io.vproxy.pni.PNIEnv;
import io.vproxy.pni.PNILinkOptions;
import io.vproxy.pni.PanamaUtils;

import java.lang.foreign.MemorySegment;
import java.lang.invoke.MethodHandle;

/**
 * Downcalls into libvpcsum.so (MI355X batched Internet checksum), written in the shape the PNI
 * generator emits for the existing natives (compare
 * base/src/main/generated/io/vproxy/vfd/posix/PosixNative.java:729-744 in vproxy): one
 * downcall per method, exceptions travel through the PNIEnv (0 = ok, -1 = exception stored in
 * ENV).  The C side is include/vpcsum.h, symbols Java_io_vproxy_vpcsum_VPCsum_*.
 *
 * No method is linked critical ({@code setCritical(false)} throughout): every entry point may
 * block -- create / registerArena allocate and page-lock through the HIP runtime, submit / submitPre /
 * natSubmit / verifyFrames / parseFrames finish the batch that last used their slot (an event wait, or the
 * service grid's completion), waitFor and setService wait by design.  A critical downcall keeps
 * the thread in Java state and would stall every safepoint (GC included) for that long.
 *
 * Load the library the same way vproxy loads its other natives:
 * {@code Utils.loadDynamicLibrary("vpcsum")} (base/src/main/java/io/vproxy/base/util/Utils.java:1014-1030).
 *
 * Not compiled in this repository (the build image has no JDK); see INTEGRATION.md.
 */
public class VPCsum {
    private VPCsum() {
    }

    private static final VPCsum INSTANCE = new VPCsum();

    public static VPCsum get() {
        return INSTANCE;
    }

    /** include/vpcsum.h VPCSUM_ABI_VERSION this binding was written against (4: the ingress header
     * sum, verifyFramesHsum and PRE_HSUM entries; 3: VPCSUM_F_PRE and submitPre; 2: NAT_DEC_TTL
     * refuses TTL <= 1 with S_TTL_EXPIRED).  {@link #abiVersion} reports the loaded library's. */
    public static final int ABI_VERSION = 4;

    /** vpcsum_abi_version() of the loaded library (a plain C function, no PNIEnv; {@link VPCsumLib}).
     * Throws an IOException when libvpcsum is not loaded. */
    public int abiVersion() throws java.io.IOException {
        return VPCsumLib.abiVersion();
    }

    // descriptor flags (include/vpcsum.h)
    public static final int F_IP = 0x01;
    public static final int F_L4 = 0x02;
    public static final int F_RAW = 0x04;
    /** checksum offload (VP_CSUM_UP_PSEUDO): L4 field = folded pseudo-header sum (CHECKSUM_PARTIAL) */
    public static final int F_L4P = 0x08;
    /** a received packet changed in place whose stored L4 sum was verified on ingress: its L4 sum
     * is updated from its pre-image entry by RFC 1624 -- only the header is read ({@link PreImage}) */
    public static final int F_PRE = 0x10;
    /** bytes of one vpcsum_pre_t pre-image entry (the vpcsum_nat_t layout) */
    public static final int PRE_ENTRY = 48;
    /** pre-image entry mask: the entry's first 8 bytes hold the frame's ingress header sum
     * (vpcsum_hsum_t, {@link #verifyFramesHsum}) */
    public static final int PRE_HSUM = 0x80;
    /** bytes of one vpcsum_hsum_t: sum(u16) l4Len(u16) hlen proto ver l2Len */
    public static final int HSUM_ENTRY = 8;
    // status bits
    public static final int S_IP_OK = 0x01;
    public static final int S_L4_OK = 0x02;
    public static final int S_UDP_NOCSUM = 0x04;
    public static final int S_DONE = 0x40;
    public static final int S_BAD_DESC = 0x80;
    /** NAT: a TTL / hop-limit decrement of a packet at TTL <= 1 is refused (with S_BAD_DESC);
     * IPInputRoute drops such packets and answers ICMP time exceeded (IPInputRoute.java:81-88). */
    public static final int S_TTL_EXPIRED = 0x20;
    // modes
    public static final int MODE_COMPUTE = 0x00;
    public static final int MODE_VERIFY = 0x01;
    public static final int MODE_WRITE = 0x10;
    // NAT / TTL rewrite masks (vpcsum_nat_t.mask) and modes
    public static final int NAT_SRC = 0x01;
    public static final int NAT_DST = 0x02;
    public static final int NAT_SPORT = 0x04;
    public static final int NAT_DPORT = 0x08;
    public static final int NAT_DEC_TTL = 0x10;
    public static final int NAT_SET_TTL = 0x20;
    public static final int NAT_RFC1624 = 0x00;
    public static final int NAT_STRICT_JAVA = 0x01;
    /** bytes of one vpcsum_nat_t rewrite entry: src[16] dst[16] sport[2] dport[2] mask ttl rsv[10] */
    public static final int NAT_ENTRY = 48;

    private static final MethodHandle createMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_create", int.class /* device */, long.class /* maxArena */, int.class /* maxPkts */);

    /** Create a context on GPU {@code device}: device buffers for one batch of up to maxPkts
     * packets spanning at most maxArena bytes (double buffered). Returns an opaque handle. */
    public long create(PNIEnv ENV, int device, long maxArena, int maxPkts) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) createMH.invokeExact(ENV.MEMORY, device, maxArena, maxPkts);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
        return ENV.returnLong();
    }

    private static final MethodHandle registerArenaMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_registerArena", long.class /* ctx */, MemorySegment.class /* arena */, long.class /* len */);

    /** Page-lock a long-lived arena (an AF_XDP umem, UMem.java:36-44) once, so batches from it
     * DMA straight to the GPU without a staging copy. */
    public void registerArena(PNIEnv ENV, long ctx, MemorySegment arena, long len) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) registerArenaMH.invokeExact(ENV.MEMORY, ctx, arena, len);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
    }

    private static final MethodHandle submitMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_submit", long.class /* ctx */, MemorySegment.class /* arena */, long.class /* arenaLen */,
        MemorySegment.class /* desc */, int.class /* n */, MemorySegment.class /* out */, MemorySegment.class /* status */,
        int.class /* mode */);

    /** Asynchronously checksum n packets described by 16-byte descriptors (vpcsum_desc_t) over
     * {@code arena}. Returns a ticket for {@link #waitFor}. */
    public long submit(PNIEnv ENV, long ctx, MemorySegment arena, long arenaLen, MemorySegment desc, int n,
                       MemorySegment out, MemorySegment status, int mode) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) submitMH.invokeExact(ENV.MEMORY, ctx, arena, arenaLen, desc, n, out, status, mode);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
        return ENV.returnLong();
    }

    private static final MethodHandle submitPreMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_submitPre", long.class /* ctx */, MemorySegment.class /* arena */,
        long.class /* arenaLen */, MemorySegment.class /* desc */, MemorySegment.class /* pre */, int.class /* n */,
        MemorySegment.class /* out */, MemorySegment.class /* status */, int.class /* mode */);

    /** {@link #submit} for an egress batch that holds frames changed in place: descriptors with
     * F_PRE take their L4 sum from {@code pre[i]} (48-B vpcsum_pre_t: a PRE_HSUM entry,
     * {@link PreImage#writeTo}) by RFC 1624, reading only the frame's header; the others are summed
     * in full (vpcsum_ctx_submit_pre).  mode: MODE_COMPUTE or MODE_WRITE.  Returns a ticket for
     * {@link #waitFor}. */
    public long submitPre(PNIEnv ENV, long ctx, MemorySegment arena, long arenaLen, MemorySegment desc, MemorySegment pre,
                          int n, MemorySegment out, MemorySegment status, int mode) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) submitPreMH.invokeExact(ENV.MEMORY, ctx, arena, arenaLen, desc, pre, n, out, status, mode);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
        return ENV.returnLong();
    }

    private static final MethodHandle waitForMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_waitFor", long.class /* ctx */, long.class /* ticket */);

    /** Block until the batch of {@code ticket} is done; results (and, with MODE_WRITE, the
     * checksum fields inside the frames) are valid afterwards. */
    public void waitFor(PNIEnv ENV, long ctx, long ticket) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) waitForMH.invokeExact(ENV.MEMORY, ctx, ticket);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
    }

    private static final MethodHandle verifyFramesMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_verifyFrames", long.class /* ctx */, MemorySegment.class /* arena */,
        long.class /* arenaLen */, MemorySegment.class /* frameOff */, MemorySegment.class /* frameLen */, int.class /* n */,
        MemorySegment.class /* out */, MemorySegment.class /* status */);

    /** Ingress verify of a received batch: the raw Ethernet frames at frameOff[i] (u64, bytes into
     * {@code arena}, which must be registered) of frameLen[i] (u32) bytes are parsed on the GPU with
     * the rules of EthernetPacket/Ipv4Packet/Ipv6Packet.from and verified where they lie.
     * status[i] gets S_IP_OK / S_L4_OK / S_UDP_NOCSUM (or S_BAD_DESC when the frame does not parse).
     * Returns a ticket for {@link #waitFor}. */
    public long verifyFrames(PNIEnv ENV, long ctx, MemorySegment arena, long arenaLen, MemorySegment frameOff,
                             MemorySegment frameLen, int n, MemorySegment out, MemorySegment status) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) verifyFramesMH.invokeExact(ENV.MEMORY, ctx, arena, arenaLen, frameOff, frameLen, n, out, status);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
        return ENV.returnLong();
    }

    private static final MethodHandle verifyFramesHsumMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_verifyFramesHsum", long.class /* ctx */, MemorySegment.class /* arena */,
        long.class /* arenaLen */, MemorySegment.class /* frameOff */, MemorySegment.class /* frameLen */, int.class /* n */,
        MemorySegment.class /* out */, MemorySegment.class /* status */, MemorySegment.class /* hsum */);

    /** {@link #verifyFrames} that also records each frame's ingress header sum: hsum[i] (8 B,
     * vpcsum_hsum_t: the sum of the L4 sum's words the in-place setters can reach, the segment and
     * header lengths, protocol, version and the L3 offset in the frame; all zero for a frame without
     * one).  The egress flush of a frame changed in place updates its L4 sum from it
     * ({@link GpuCsumBatch#defer}, INTEGRATION.md §5).  Returns a ticket for {@link #waitFor}. */
    public long verifyFramesHsum(PNIEnv ENV, long ctx, MemorySegment arena, long arenaLen, MemorySegment frameOff,
                                 MemorySegment frameLen, int n, MemorySegment out, MemorySegment status,
                                 MemorySegment hsum) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) verifyFramesHsumMH.invokeExact(ENV.MEMORY, ctx, arena, arenaLen, frameOff, frameLen, n, out, status,
                                                       hsum);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
        return ENV.returnLong();
    }

    private static final MethodHandle parseFramesMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_parseFrames", long.class /* ctx */, MemorySegment.class /* arena */,
        long.class /* arenaLen */, MemorySegment.class /* frameOff */, MemorySegment.class /* frameLen */, int.class /* n */,
        MemorySegment.class /* desc */, MemorySegment.class /* status */, MemorySegment.class /* tuples */);

    /** Batched parse of a received batch with flow tuples: the frames at frameOff[i] / frameLen[i]
     * of the registered {@code arena} are parsed on the GPU (EthernetPacket/Ipv4Packet/Ipv6Packet
     * rules).  After {@link #waitFor}: desc[i] (16 B, ready for submit / natSubmit), status[i]
     * (0 or S_BAD_DESC) and tuples[i] (40 B: src[16] dst[16] sport[2] dport[2] ver proto
     * tcpFlags rsv, network order), the key TcpInput / UdpInput look up in the conntrack
     * (TcpInput.java:47-51, UdpInput.java:45-47).  Returns a ticket. */
    public long parseFrames(PNIEnv ENV, long ctx, MemorySegment arena, long arenaLen, MemorySegment frameOff,
                            MemorySegment frameLen, int n, MemorySegment desc, MemorySegment status,
                            MemorySegment tuples) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) parseFramesMH.invokeExact(ENV.MEMORY, ctx, arena, arenaLen, frameOff, frameLen, n, desc, status, tuples);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
        return ENV.returnLong();
    }

    private static final MethodHandle egressFramesMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_egressFrames", long.class /* ctx */, MemorySegment.class /* arena */,
        long.class /* arenaLen */, MemorySegment.class /* frameOff */, MemorySegment.class /* frameLen */,
        MemorySegment.class /* frameFlags */, int.class /* n */, MemorySegment.class /* out */,
        MemorySegment.class /* status */);

    /** Egress flush straight from the frames: frameOff[i] (u64) / frameLen[i] (u32) as the TX ring
     * sends them, frameFlags[i] (u8) the F_* sums each needs.  The GPU parses every frame with the
     * vswitch's rules and writes its sums in place, in one submission; after {@link #waitFor}
     * status[i] is S_DONE or S_BAD_DESC (refused, nothing written: hand the frame back).
     * Returns a ticket. */
    public long egressFrames(PNIEnv ENV, long ctx, MemorySegment arena, long arenaLen, MemorySegment frameOff,
                             MemorySegment frameLen, MemorySegment frameFlags, int n, MemorySegment out,
                             MemorySegment status) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) egressFramesMH.invokeExact(ENV.MEMORY, ctx, arena, arenaLen, frameOff, frameLen, frameFlags, n,
                                                   out, status);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
        return ENV.returnLong();
    }

    private static final MethodHandle natSubmitMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_natSubmit", long.class /* ctx */, MemorySegment.class /* arena */,
        long.class /* arenaLen */, MemorySegment.class /* desc */, MemorySegment.class /* rw */, int.class /* n */,
        MemorySegment.class /* status */, int.class /* natMode */);

    /** SwitchUtils.applyNat for a batch (SwitchUtils.java:522-542): rewrite {@code rw[i]}
     * (48-byte vpcsum_nat_t entries: addresses, ports, TTL / hop limit) into the packet of
     * {@code desc[i]} in place, with the checksums updated as getRawPacket(0) would recompute them
     * (NAT_RFC1624 on valid input, NAT_STRICT_JAVA for any input).  Frames in the registered umem
     * are rewritten where they lie.  status[i]: S_DONE or S_BAD_DESC.  Returns a ticket for
     * {@link #waitFor}. */
    public long natSubmit(PNIEnv ENV, long ctx, MemorySegment arena, long arenaLen, MemorySegment desc,
                          MemorySegment rw, int n, MemorySegment status, int natMode) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) natSubmitMH.invokeExact(ENV.MEMORY, ctx, arena, arenaLen, desc, rw, n, status, natMode);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
        return ENV.returnLong();
    }

    private static final MethodHandle setServiceMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_setService", long.class /* ctx */, int.class /* idleUs */);

    /** Low-latency flushes: batches of up to 512 packets from a registered arena go to a resident
     * GPU grid that polls a pinned mailbox, instead of a kernel launch each (about 13 us for 32
     * frames instead of 19).  The grid leaves after {@code idleUs} without a batch and restarts on
     * the next submit; 0 turns it off.  It waits for batches in flight. */
    public void setService(PNIEnv ENV, long ctx, int idleUs) throws java.io.IOException {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) setServiceMH.invokeExact(ENV.MEMORY, ctx, idleUs);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwIf(java.io.IOException.class);
            ENV.throwLast();
        }
    }

    private static final MethodHandle closeMH = PanamaUtils.lookupPNIFunction(new PNILinkOptions().setCritical(false),
        "Java_io_vproxy_vpcsum_VPCsum_close", long.class /* ctx */);

    public void close(PNIEnv ENV, long ctx) {
        ENV.reset();
        int ERR;
        try {
            ERR = (int) closeMH.invokeExact(ENV.MEMORY, ctx);
        } catch (Throwable THROWABLE) {
            throw PanamaUtils.convertInvokeExactException(THROWABLE);
        }
        if (ERR != 0) {
            ENV.throwLast();
        }
    }
}
