package io.vproxy.vpcsum;

import io.vproxy.pni.PNIEnv;
import io.vproxy.vpacket.AbstractIpPacket;
import io.vproxy.vpacket.EthernetPacket;
import io.vproxy.vpacket.IcmpPacket;
import io.vproxy.vpacket.Ipv4Packet;
import io.vproxy.vpacket.Ipv6Packet;
import io.vproxy.vpxdp.ChunkInfo;
import io.vproxy.vpxdp.XDPConsts;
import io.vproxy.vswitch.PacketBuffer;

import java.io.IOException;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.ValueLayout;

/**
 * Egress / ingress checksum batch for ONE umem (AF_XDP frame arena) and ONE switch event loop.
 *
 * Egress is the flag-and-flush contract the XDP path already has with its native code
 * (SwitchUtils.checksumFlagsFor, SwitchUtils.java:297-316; XDPIface.sendPacket / completeTx,
 * XDPIface.java:100-178, 227-243): {@link #defer} takes over the VP_CSUM_* work of a frame instead
 * of leaving it to the native path, {@link #flush} (called at the top of Iface.completeTx, before
 * xsk.writePackets) computes every deferred sum in one GPU pass (the resident service grid for
 * flushes of up to 512 frames, a launch above that) and writes the results into the frames
 * (MODE_WRITE), byte-for-byte what getRawPacket(0) would have produced
 * (AbstractPacket.java:15-22 -> Ipv4Packet.__updateChecksum :209-217, TcpPacket/UdpPacket/IcmpPacket
 * updateChecksumWith*).
 *
 * Ingress verify (new capability, SURVEY.md §8(a) A11): {@link #verify} fills one status byte per
 * frame of a received batch (XDPIface.readable, XDPIface.java:281-314).
 *
 * One instance per event loop: like everything on the vswitch data path it is single-threaded
 * (Switch.java:170-199).  Not compiled in this repository (no JDK in the build image).
 *
 * The status segment that {@link #nat}, {@link #verify} and {@link #verifyFrames} return is this
 * instance's own buffer: it is valid until the next call on this instance (the next flush, NAT or
 * verify overwrites it).  Copy what must outlive that, or pass your own segment to the overloads
 * that take one.
 *
 * Received frames changed in place (INTEGRATION.md §5): {@link #verifyFrames} records each frame's
 * ingress header sum with its status ({@link PreImage#received}); {@link #defer} marks a frame F_PRE
 * when {@link PreImage#eligible} holds -- verified L4 sum, the received frame leaving in place, the
 * record's lengths -- and the flush updates its L4 sum from the record and the header words now in
 * the frame, whatever the setters changed there (NAT, the PROXY-protocol SYN rewrite, an MSS clamp),
 * reading only the header (VPCsum.submitPre).  Otherwise the frame is summed in full, like Java's
 * getRawPacket(0).
 *
 * {@link #stats} counts where every deferred frame went (GPU, small-flush hand-back, rejected
 * descriptor hand-back), next to IfaceStatistics: with INTEGRATION.md §3's diff the interface keeps
 * counting csum_skip for every frame whose sums Java left to someone else, the GPU included.
 */
public final class GpuCsumBatch implements AutoCloseable {
    private static final int DESC = 16;

    private final PNIEnv env = new PNIEnv();
    private final long ctx;
    private final MemorySegment umem;
    private final long umemLen;
    private final Arena arena = Arena.ofShared();
    private final MemorySegment desc;
    private final MemorySegment pre;      // pre-images of the F_PRE frames (48 B per descriptor slot)
    private final MemorySegment hsum;     // ingress header sums of the last verified RX batch (8 B per frame)
    private int nPre = 0;                 // F_PRE frames in the pending descriptor batch
    private final MemorySegment out;
    private final MemorySegment status;
    private final int capacity;
    private final ChunkInfo[] chunks;
    private final int[] nativeFlagsOf;
    private int n = 0;
    // deferFrame: raw frames whose descriptors the GPU builds itself (VPCsum.egressFrames)
    private final MemorySegment frameOff;
    private final MemorySegment frameLen;
    private final MemorySegment frameFlags;
    private final ChunkInfo[] frameChunks;
    private final int[] frameNativeFlags;
    private int nFrames = 0;

    /** Where the deferred frames went (cumulative).  Invariant after a flush:
     * deferred == gpuHandled + smallFlushHandedBack + badDescHandedBack. */
    public static final class Stats {
        public long deferred;              // frames taken over by defer / deferFrame
        public long gpuHandled;            // frames the GPU wrote
        public long smallFlushHandedBack;  // frames of flushes below SMALL_FLUSH, back to vpxdp
        public long badDescHandedBack;     // frames the kernel refused (S_BAD_DESC), back to vpxdp
        public long gpuFlushes;            // flushes that went to the GPU
        public long preDeferred;           // received frames updated from their header sum (F_PRE, header only)
        public long preFull;               // received frames with a record that took the full recompute
                                           // (no verified L4 sum, rebuilt, moved, other lengths)

        @Override
        public String toString() {
            return "csum_deferred=" + deferred + " csum_gpu=" + gpuHandled + " csum_small_flush=" + smallFlushHandedBack
                   + " csum_bad_desc=" + badDescHandedBack + " csum_gpu_flushes=" + gpuFlushes
                   + " csum_pre=" + preDeferred + " csum_pre_full=" + preFull;
        }
    }

    private final Stats stats = new Stats();

    public Stats stats() {
        return stats;
    }

    /** Flushes of fewer frames go back to the native VP_CSUM_* path (the GPU breaks even at about
     * 5 frames per flush with the service grid, DESIGN.md §8). */
    public static final int SMALL_FLUSH = 5;

    public GpuCsumBatch(int device, MemorySegment umem, int capacity) throws IOException {
        this.umem = umem;
        this.umemLen = umem.byteSize();
        this.capacity = capacity;
        // before VPCsum is initialised (its PNI handles resolve in its static initialiser): a missing
        // library or another ABI is an IOException here (VPCsum.ABI_VERSION is a constant: reading
        // it does not initialise the class)
        VPCsumLib.requireAbi(VPCsum.ABI_VERSION);
        this.ctx = VPCsum.get().create(env, device, umemLen, capacity);
        VPCsum.get().registerArena(env, ctx, umem, umemLen);
        // completeTx flushes are small: keep a resident GPU grid polling for them (20 ms idle).
        // Until it leaves, that grid is device work: a hipDeviceSynchronize or hipFree by another
        // user of this GPU in this process waits up to 20 ms for it (INTEGRATION.md §7)
        VPCsum.get().setService(env, ctx, 20_000);
        this.desc = arena.allocate((long) DESC * capacity, 16);
        this.pre = arena.allocate((long) VPCsum.PRE_ENTRY * capacity, 16);
        this.hsum = arena.allocate((long) VPCsum.HSUM_ENTRY * capacity, 16);
        this.out = arena.allocate(4L * capacity, 16);
        this.status = arena.allocate(capacity, 16);
        this.chunks = new ChunkInfo[capacity];
        this.nativeFlagsOf = new int[capacity];
        this.frameOff = arena.allocate(8L * capacity, 16);
        this.frameLen = arena.allocate(4L * capacity, 16);
        this.frameFlags = arena.allocate(capacity, 16);
        this.frameChunks = new ChunkInfo[capacity];
        this.frameNativeFlags = new int[capacity];
    }

    /**
     * The alternative to {@link #defer}: nothing is read from the Java packet objects.  The frame
     * is handed over as XDPIface.sendPacket already has it -- its umem offset {@code pktaddr}
     * (chunk.getAddr() + pkb.pktOff, or the copy's address) and {@code pktlen}
     * (pkb.pktBuf.length(), Ethernet padding included) -- with the sums checksumFlagsFor asked for,
     * and the GPU parses it with the vswitch's rules (L3 after the Ethernet / 802.1Q header,
     * lengths from totalLength / payloadLength, L4 after IHL or the extension header) before it
     * writes the sums (vpcsum_ctx_egress_frames).  Returns the flags the chunk keeps, as
     * {@link #defer}; a frame the GPU refuses gets its native flags back at {@link #flush}.
     */
    public int deferFrame(ChunkInfo chunk, long pktaddr, int pktlen, int nativeFlags) {
        int flags = 0;
        int keep = nativeFlags & XDPConsts.VP_CSUM_XDP_OFFLOAD;
        if ((nativeFlags & XDPConsts.VP_CSUM_IP) != 0) flags |= VPCsum.F_IP;
        if ((nativeFlags & XDPConsts.VP_CSUM_UP) != 0) flags |= VPCsum.F_L4;
        // the GPU refuses F_L4P for an ICMPv4 message (no pseudo header) and hands it back whole
        if ((nativeFlags & XDPConsts.VP_CSUM_UP_PSEUDO) != 0) flags |= VPCsum.F_L4P;
        if (flags == 0) {
            return nativeFlags;
        }
        if (nFrames == capacity) {
            throw new IllegalStateException("batch full: flush first");
        }
        frameOff.setAtIndex(ValueLayout.JAVA_LONG, nFrames, pktaddr);
        frameLen.setAtIndex(ValueLayout.JAVA_INT, nFrames, pktlen);
        frameFlags.set(ValueLayout.JAVA_BYTE, nFrames, (byte) flags);
        frameChunks[nFrames] = chunk;
        frameNativeFlags[nFrames] = nativeFlags;
        ++nFrames;
        ++stats.deferred;
        return keep;
    }

    public boolean isFull() {
        return n == capacity || nFrames == capacity;
    }

    /**
     * Take over the dirty checksums of {@code pkb}, whose Ethernet frame lies in the umem at byte
     * offset {@code frameAddr} in {@code chunk} (the zero-copy branch of XDPIface.sendPacket:
     * chunk.getAddr() + pkb.pktOff; the copying branch: the pktaddr the frame was copied to).
     * {@code nativeFlags} is what SwitchUtils.checksumFlagsFor (SwitchUtils.java:297-316) returned
     * for the packet: VP_CSUM_IP -> F_IP, VP_CSUM_UP -> F_L4, VP_CSUM_UP_PSEUDO -> F_L4P (the GPU
     * writes the pseudo-header sum, the NIC completes it; an ICMPv4 message has no pseudo header,
     * so it stays with the native path).  Returns the flags the chunk must carry now:
     * VP_CSUM_XDP_OFFLOAD (and the ICMPv4 pseudo request) stay, the rest is the GPU's.  A flush
     * below {@link #SMALL_FLUSH} frames hands every deferred frame back to the native path instead
     * (its full nativeFlags are restored on the chunk): a GPU round trip costs more than the CPU
     * there (DESIGN.md §8).
     */
    public int defer(PacketBuffer pkb, ChunkInfo chunk, long frameAddr, int nativeFlags) {
        if (nativeFlags == 0 || !(pkb.pkt.getPacket() instanceof AbstractIpPacket ip)) {
            return nativeFlags;
        }
        int flags = 0;
        int keep = nativeFlags & XDPConsts.VP_CSUM_XDP_OFFLOAD;
        if ((nativeFlags & XDPConsts.VP_CSUM_IP) != 0) {
            flags |= VPCsum.F_IP;
        }
        if ((nativeFlags & XDPConsts.VP_CSUM_UP) != 0) {
            flags |= VPCsum.F_L4;
        }
        if ((nativeFlags & XDPConsts.VP_CSUM_UP_PSEUDO) != 0) {
            if (ip.getPacket() instanceof IcmpPacket icmp && !icmp.isIpv6()) {
                keep |= XDPConsts.VP_CSUM_UP_PSEUDO;
            } else {
                flags |= VPCsum.F_L4P;
            }
        }
        if (flags == 0) {
            return nativeFlags;
        }
        if (n == capacity) {
            throw new IllegalStateException("batch full: flush first");
        }
        long l3 = frameAddr + (((EthernetPacket) pkb.pkt).getVlan() >= 0 ? 18 : 14);
        // The lengths come from the IP header fields, never from the buffer: a frame parsed with
        // allowPartial (every XDP / tap frame, PacketBuffer.java:177 -> EthernetPacket.java:52-56)
        // keeps its Ethernet padding in pktBuf (Ipv4Packet.initPartial does not cut it,
        // Ipv4Packet.java:29-63) and leaves `options` empty, so getRawPacket().length() counts the
        // padding of every 60-B frame and getHeaderSize() is 20 for any IHL.  Java's own recompute
        // covers raw.sub(ihl*4, totalLength - ihl*4) (:55).
        int l3len;
        int l4off;
        if (ip instanceof Ipv4Packet v4) {
            l3len = v4.getTotalLength();           // Ipv4Packet.java:361
            l4off = v4.getIhl() * 4;               // :334
        } else {
            Ipv6Packet v6 = (Ipv6Packet) ip;
            l3len = 40 + v6.getPayloadLength();    // Ipv6Packet.java:332
            l4off = v6.getHeaderSize();            // :427-435, extHeaders filled by from() (:33-35)
        }
        int ver = ip instanceof Ipv4Packet ? 4 : 6;
        // a received frame changed in place whose stored L4 sum the ingress verify proved: its L4
        // sum is updated from its ingress header sum, only its header read (PreImage)
        if ((flags & VPCsum.F_L4) != 0 && pkb.csumHsum != 0) {
            if (PreImage.eligible(pkb, chunk, umem, l3, ver, ip.getProtocol(), l3len, l4off)) {
                flags |= VPCsum.F_PRE;
                PreImage.writeTo(pre, (long) VPCsum.PRE_ENTRY * n, pkb.csumHsum);
                ++nPre;
                ++stats.preDeferred;
            } else {
                ++stats.preFull;
            }
        }
        long d = (long) DESC * n;
        desc.set(ValueLayout.JAVA_LONG_UNALIGNED, d, l3);
        desc.set(ValueLayout.JAVA_SHORT_UNALIGNED, d + 8, (short) l3len);
        desc.set(ValueLayout.JAVA_SHORT_UNALIGNED, d + 10, (short) l4off);
        desc.set(ValueLayout.JAVA_BYTE, d + 12, (byte) ver);
        desc.set(ValueLayout.JAVA_BYTE, d + 13, (byte) ip.getProtocol());
        desc.set(ValueLayout.JAVA_BYTE, d + 14, (byte) flags);
        desc.set(ValueLayout.JAVA_BYTE, d + 15, (byte) 0);
        chunks[n] = chunk;
        nativeFlagsOf[n] = nativeFlags;
        ++n;
        ++stats.deferred;
        return keep;
    }

    /**
     * Compute and write every deferred checksum into its frame; call at the top of
     * Iface.completeTx, before xsk.writePackets.  Returns the frames the GPU handled (0 when a
     * small flush went back to the native path).  A frame whose descriptor the kernel rejected
     * (S_BAD_DESC: nothing was written) gets its native VP_CSUM_* flags back, so the native path
     * computes its sums at xsk.writePackets instead of the frame leaving with a stale checksum.
     */
    public int flush() throws IOException {
        return flushDescriptors() + flushFrames();
    }

    private int flushFrames() throws IOException {
        if (nFrames == 0) {
            return 0;
        }
        int done = nFrames;
        if (nFrames < SMALL_FLUSH) {
            for (int i = 0; i < nFrames; ++i) {
                frameChunks[i].setCsumFlags(frameNativeFlags[i]);
                frameChunks[i] = null;
            }
            stats.smallFlushHandedBack += nFrames;
            nFrames = 0;
            return 0;
        }
        long t = VPCsum.get().egressFrames(env, ctx, umem, umemLen, frameOff, frameLen, frameFlags, nFrames, out, status);
        VPCsum.get().waitFor(env, ctx, t);
        for (int i = 0; i < nFrames; ++i) {
            if ((status.get(ValueLayout.JAVA_BYTE, i) & VPCsum.S_BAD_DESC) != 0) {
                frameChunks[i].setCsumFlags(frameNativeFlags[i]);
                --done;
            }
            frameChunks[i] = null;
        }
        stats.gpuHandled += done;
        stats.badDescHandedBack += nFrames - done;
        ++stats.gpuFlushes;
        nFrames = 0;
        return done;
    }

    private int flushDescriptors() throws IOException {
        if (n == 0) {
            return 0;
        }
        int done = n;
        if (n < SMALL_FLUSH) {
            for (int i = 0; i < n; ++i) {
                chunks[i].setCsumFlags(nativeFlagsOf[i]);
                chunks[i] = null;
            }
            stats.smallFlushHandedBack += n;
            n = 0;
            nPre = 0;
            return 0;
        }
        long t = nPre > 0 ? VPCsum.get().submitPre(env, ctx, umem, umemLen, desc, pre, n, out, status, VPCsum.MODE_WRITE)
                          : VPCsum.get().submit(env, ctx, umem, umemLen, desc, n, out, status, VPCsum.MODE_WRITE);
        nPre = 0;
        VPCsum.get().waitFor(env, ctx, t);
        for (int i = 0; i < n; ++i) {
            if ((status.get(ValueLayout.JAVA_BYTE, i) & VPCsum.S_BAD_DESC) != 0) {
                chunks[i].setCsumFlags(nativeFlagsOf[i]);
                --done;
            }
            chunks[i] = null;
        }
        stats.gpuHandled += done;
        stats.badDescHandedBack += n - done;
        ++stats.gpuFlushes;
        n = 0;
        return done;
    }

    /**
     * SwitchUtils.applyNat for a batch of frames in the umem (SwitchUtils.java:522-542): each
     * 48-byte entry of {@code rw} (addresses, ports, TTL / hop limit; VPCsum.NAT_*) rewrites the
     * packet of the matching descriptor of {@code natDesc} in place, checksums updated as the
     * setters + getRawPacket(0) would leave them.  Returns one status byte per packet in this
     * instance's status segment, valid until the next call on this instance (see the class note).
     */
    public MemorySegment nat(MemorySegment natDesc, MemorySegment rw, int count, boolean strictJava) throws IOException {
        return nat(natDesc, rw, count, strictJava, status);
    }

    /** {@link #nat} with the status bytes written to the caller's {@code statusOut} (count bytes). */
    public MemorySegment nat(MemorySegment natDesc, MemorySegment rw, int count, boolean strictJava,
                             MemorySegment statusOut) throws IOException {
        long t = VPCsum.get().natSubmit(env, ctx, umem, umemLen, natDesc, rw, count, statusOut,
            strictJava ? VPCsum.NAT_STRICT_JAVA : VPCsum.NAT_RFC1624);
        VPCsum.get().waitFor(env, ctx, t);
        return statusOut;
    }

    /**
     * Ingress verify of {@code count} frames already described in {@code desc} (e.g. built by the
     * GPU parser, vpcsum_parse_ether_async): fills {@code status} (S_IP_OK / S_L4_OK /
     * S_UDP_NOCSUM per frame) without touching the frames.  The returned segment is this
     * instance's, valid until the next call on it (see the class note).
     */
    public MemorySegment verify(MemorySegment frameDesc, int count) throws IOException {
        return verify(frameDesc, count, status);
    }

    /** {@link #verify} with the status bytes written to the caller's {@code statusOut} (count bytes). */
    public MemorySegment verify(MemorySegment frameDesc, int count, MemorySegment statusOut) throws IOException {
        long t = VPCsum.get().submit(env, ctx, umem, umemLen, frameDesc, count, MemorySegment.NULL, statusOut, VPCsum.MODE_VERIFY);
        VPCsum.get().waitFor(env, ctx, t);
        return statusOut;
    }

    /**
     * Ingress verify straight from the RX ring (XDPIface.readable, XDPIface.java:281-314): the
     * {@code count} received frames at umem offsets {@code frameOff} (u64 each) with lengths
     * {@code frameLen} (u32 each) are parsed and verified on the GPU in one submission, without
     * building descriptors in Java, and each frame's ingress header sum is recorded
     * ({@link #headerSums}).  Returns one status byte per frame, in this instance's segment, valid
     * until the next call on it (see the class note).  Hand both to each frame's PacketBuffer with
     * {@link PreImage#received}.
     */
    public MemorySegment verifyFrames(MemorySegment frameOff, MemorySegment frameLen, int count) throws IOException {
        return verifyFrames(frameOff, frameLen, count, status, hsum);
    }

    /** {@link #verifyFrames} with the status bytes and header sums (8 B per frame) written to the
     * caller's segments. */
    public MemorySegment verifyFrames(MemorySegment frameOff, MemorySegment frameLen, int count,
                                      MemorySegment statusOut, MemorySegment hsumOut) throws IOException {
        // no out words: the status bytes are the ingress result (writing the sums too cost verify 4%
        // on 64-B frames, DESIGN.md §5)
        long t = VPCsum.get().verifyFramesHsum(env, ctx, umem, umemLen, frameOff, frameLen, count, MemorySegment.NULL,
                                               statusOut, hsumOut);
        VPCsum.get().waitFor(env, ctx, t);
        return statusOut;
    }

    /** The header sums of the last {@link #verifyFrames} batch (8 B per frame), valid until the next
     * verify on this instance. */
    public MemorySegment headerSums() {
        return hsum;
    }

    /**
     * Parse of a received batch with flow tuples (XDPIface.readable, then TcpInput / UdpInput's
     * conntrack lookups, TcpInput.java:47-51, UdpInput.java:45-47): {@code count} frames at umem
     * offsets {@code frameOff} (u64) with lengths {@code frameLen} (u32).  Fills {@code desc}
     * (16 B per frame, usable by {@link #nat} and {@link #verify}), {@code parseStatus} (0 or
     * S_BAD_DESC) and {@code tuples} (40 B per frame).
     */
    public void parseFrames(MemorySegment frameOff, MemorySegment frameLen, int count, MemorySegment desc,
                            MemorySegment parseStatus, MemorySegment tuples) throws IOException {
        long t = VPCsum.get().parseFrames(env, ctx, umem, umemLen, frameOff, frameLen, count, desc, parseStatus, tuples);
        VPCsum.get().waitFor(env, ctx, t);
    }

    @Override
    public void close() {
        VPCsum.get().close(env, ctx);
        arena.close();
    }
}
