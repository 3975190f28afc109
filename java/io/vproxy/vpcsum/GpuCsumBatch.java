package io.vproxy.vpcsum;

import io.vproxy.pni.PNIEnv;
import io.vproxy.vpacket.AbstractIpPacket;
import io.vproxy.vpacket.EthernetPacket;
import io.vproxy.vpacket.IcmpPacket;
import io.vproxy.vpacket.Ipv4Packet;
import io.vproxy.vpacket.TcpPacket;
import io.vproxy.vpacket.UdpPacket;
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
 * XDPIface.java:100-178, 227-243): {@link #defer} records which sums of a frame are dirty instead
 * of setting VP_CSUM_* on the chunk, {@link #flush} (called at the top of Iface.completeTx, before
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
 */
public final class GpuCsumBatch implements AutoCloseable {
    private static final int DESC = 16;

    private final PNIEnv env = new PNIEnv();
    private final long ctx;
    private final MemorySegment umem;
    private final long umemLen;
    private final Arena arena = Arena.ofShared();
    private final MemorySegment desc;
    private final MemorySegment out;
    private final MemorySegment status;
    private final int capacity;
    private int n = 0;

    public GpuCsumBatch(int device, MemorySegment umem, int capacity) throws IOException {
        this.umem = umem;
        this.umemLen = umem.byteSize();
        this.capacity = capacity;
        this.ctx = VPCsum.get().create(env, device, umemLen, capacity);
        VPCsum.get().registerArena(env, ctx, umem, umemLen);
        // completeTx flushes are small: keep a resident GPU grid polling for them (20 ms idle)
        VPCsum.get().setService(env, ctx, 20_000);
        this.desc = arena.allocate((long) DESC * capacity, 16);
        this.out = arena.allocate(4L * capacity, 16);
        this.status = arena.allocate(capacity, 16);
    }

    public boolean isFull() {
        return n == capacity;
    }

    /**
     * Record the dirty checksums of {@code pkb}, whose frame lies in the umem at byte offset
     * {@code frameOff} (chunk address + pkb.pktOff).  Returns false when nothing is dirty (the
     * caller then sends the frame as is), true when the frame is now owned by the batch until
     * {@link #flush}.  Mirrors SwitchUtils.checksumFlagsFor: IP dirty -> VP_CSUM_IP, upper layer
     * dirty -> VP_CSUM_UP.
     */
    public boolean defer(PacketBuffer pkb, long frameOff) {
        return defer(pkb, frameOff, false);
    }

    /**
     * As {@link #defer(PacketBuffer, long)}; with {@code offload} (the TX queue completes L4
     * checksums: VP_CSUM_UP_PSEUDO | VP_CSUM_XDP_OFFLOAD) the upper layer gets only its
     * pseudo-header sum (F_L4P), ICMPv4 (no pseudo header) its full sum.
     */
    public boolean defer(PacketBuffer pkb, long frameOff, boolean offload) {
        if (!(pkb.pkt.getPacket() instanceof AbstractIpPacket ip)) {
            return false;
        }
        int flags = 0;
        if (ip instanceof Ipv4Packet && ip.isRequireUpdatingChecksum()) {
            flags |= VPCsum.F_IP;
        }
        // a pseudo-header change (setSrc/setDst) already marked TCP/UDP dirty through
        // pseudoHeaderChanges() (Ipv4Packet.java:236-240, Ipv6Packet.java:238-242)
        var upper = ip.getPacket();
        boolean l4Kind = upper instanceof TcpPacket || upper instanceof UdpPacket || upper instanceof IcmpPacket;
        if (l4Kind && upper.isRequireUpdatingChecksum()) {
            flags |= (offload && !(upper instanceof IcmpPacket icmp && !icmp.isIpv6())) ? VPCsum.F_L4P : VPCsum.F_L4;
        }
        if (flags == 0) {
            return false;
        }
        if (n == capacity) {
            throw new IllegalStateException("batch full: flush first");
        }
        long l3 = frameOff + (((EthernetPacket) pkb.pkt).getVlan() >= 0 ? 18 : 14);
        int l3len = ip.getRawPacket(AbstractIpPacket.FLAG_CHECKSUM_UNNECESSARY).length();
        long d = (long) DESC * n;
        desc.set(ValueLayout.JAVA_LONG_UNALIGNED, d, l3);
        desc.set(ValueLayout.JAVA_SHORT_UNALIGNED, d + 8, (short) l3len);
        desc.set(ValueLayout.JAVA_SHORT_UNALIGNED, d + 10, (short) ip.getHeaderSize());
        desc.set(ValueLayout.JAVA_BYTE, d + 12, (byte) (ip instanceof Ipv4Packet ? 4 : 6));
        desc.set(ValueLayout.JAVA_BYTE, d + 13, (byte) ip.getProtocol());
        desc.set(ValueLayout.JAVA_BYTE, d + 14, (byte) flags);
        desc.set(ValueLayout.JAVA_BYTE, d + 15, (byte) 0);
        ++n;
        return true;
    }

    /** Compute and write every deferred checksum into its frame; call before xsk.writePackets. */
    public int flush() throws IOException {
        if (n == 0) {
            return 0;
        }
        long t = VPCsum.get().submit(env, ctx, umem, umemLen, desc, n, out, status, VPCsum.MODE_WRITE);
        VPCsum.get().waitFor(env, ctx, t);
        int done = n;
        n = 0;
        return done;
    }

    /**
     * Ingress verify of {@code count} frames already described in {@code desc} (e.g. built by the
     * GPU parser, vpcsum_parse_ether_async): fills {@code status} (S_IP_OK / S_L4_OK /
     * S_UDP_NOCSUM per frame) without touching the frames.
     */
    public MemorySegment verify(MemorySegment frameDesc, int count) throws IOException {
        long t = VPCsum.get().submit(env, ctx, umem, umemLen, frameDesc, count, out, status, VPCsum.MODE_VERIFY);
        VPCsum.get().waitFor(env, ctx, t);
        return status;
    }

    /**
     * Ingress verify straight from the RX ring (XDPIface.readable, XDPIface.java:281-314): the
     * {@code count} received frames at umem offsets {@code frameOff} (u64 each) with lengths
     * {@code frameLen} (u32 each) are parsed and verified on the GPU in one submission, without
     * building descriptors in Java.  Returns one status byte per frame.
     */
    public MemorySegment verifyFrames(MemorySegment frameOff, MemorySegment frameLen, int count) throws IOException {
        long t = VPCsum.get().verifyFrames(env, ctx, umem, umemLen, frameOff, frameLen, count, out, status);
        VPCsum.get().waitFor(env, ctx, t);
        return status;
    }

    @Override
    public void close() {
        VPCsum.get().close(env, ctx);
        arena.close();
    }
}
