package io.vproxy.vpcsum;

import io.vproxy.vpacket.AbstractIpPacket;
import io.vproxy.vpacket.TcpPacket;
import io.vproxy.vpacket.TransportPacket;
import io.vproxy.vpacket.UdpPacket;
import io.vproxy.vswitch.PacketBuffer;

import java.lang.foreign.MemorySegment;
import java.lang.foreign.ValueLayout;

/**
 * The pre-image of a NAT'd packet (vpcsum_pre_t, include/vpcsum.h): the source / destination
 * address and ports as they were just before SwitchUtils.applyNat ran the setters
 * (core/.../vswitch/util/SwitchUtils.java:531-542).  At the egress flush the GPU updates the L4
 * sum from these old words and the new ones in the frame by RFC 1624, reading the frame's header
 * only, instead of summing the whole segment as getRawPacket(0) would (VPCsum.F_PRE,
 * {@link GpuCsumBatch#defer}).  That is exact when the stored L4 sum was correct before the
 * rewrite, which the ingress verify's S_L4_OK proves (PacketBuffer.csumStatus, INTEGRATION.md §5);
 * the batch falls back to the full recompute otherwise.
 *
 * One instance per PacketBuffer, reused (PacketBuffer.csumPre); {@link #record} overwrites it.
 * Not compiled in this repository (the build image has no JDK).
 */
public final class PreImage {
    private final byte[] src = new byte[16];
    private final byte[] dst = new byte[16];
    private int sport;
    private int dport;
    private int mask;
    private boolean valid;

    /**
     * Record the words applyNat's setters are about to overwrite: call it first thing in
     * SwitchUtils.applyNat (INTEGRATION.md §5).  The cached fields of the packet objects equal the
     * frame's bytes at this point (Ipv4Packet / Ipv6Packet / TcpPacket / UdpPacket.from read them
     * from the buffer, and every setter writes both).  A second NAT of the same packet keeps the
     * first record: its old words are still the ones the stored sums cover.
     */
    public static void record(PacketBuffer pkb, TransportPacket pkt) {
        if (pkb.csumPre == null) {
            pkb.csumPre = new PreImage();
        }
        PreImage p = pkb.csumPre;
        if (p.valid) {
            return;
        }
        AbstractIpPacket ip = pkb.ipPkt;
        byte[] s = ip.getSrc().getAddress();
        byte[] d = ip.getDst().getAddress();
        java.util.Arrays.fill(p.src, (byte) 0);
        java.util.Arrays.fill(p.dst, (byte) 0);
        System.arraycopy(s, 0, p.src, 0, s.length);
        System.arraycopy(d, 0, p.dst, 0, d.length);
        p.mask = VPCsum.NAT_SRC | VPCsum.NAT_DST;
        if (pkt instanceof TcpPacket || pkt instanceof UdpPacket) {
            p.sport = pkt.getSrcPort();
            p.dport = pkt.getDstPort();
            p.mask |= VPCsum.NAT_SPORT | VPCsum.NAT_DPORT;
        }
        p.valid = true;
    }

    /** Forget the record (the packet left the NAT path, or its buffer was rebuilt). */
    public void clear() {
        valid = false;
    }

    public boolean isValid() {
        return valid;
    }

    /** The 48-B vpcsum_pre_t at {@code off} of {@code seg}: src[16] dst[16] sport[2] dport[2]
     * (network order) mask, the rest 0. */
    void writeTo(MemorySegment seg, long off) {
        MemorySegment.copy(src, 0, seg, ValueLayout.JAVA_BYTE, off, 16);
        MemorySegment.copy(dst, 0, seg, ValueLayout.JAVA_BYTE, off + 16, 16);
        seg.set(ValueLayout.JAVA_BYTE, off + 32, (byte) (sport >>> 8));
        seg.set(ValueLayout.JAVA_BYTE, off + 33, (byte) sport);
        seg.set(ValueLayout.JAVA_BYTE, off + 34, (byte) (dport >>> 8));
        seg.set(ValueLayout.JAVA_BYTE, off + 35, (byte) dport);
        seg.set(ValueLayout.JAVA_BYTE, off + 36, (byte) mask);
        seg.asSlice(off + 37, 11).fill((byte) 0);
    }
}
