package io.vproxy.vpcsum;

import io.vproxy.vpxdp.ChunkInfo;
import io.vproxy.vswitch.PacketBuffer;
import io.vproxy.vswitch.util.UMemChunkByteArray;

import java.lang.foreign.MemorySegment;
import java.lang.foreign.ValueLayout;

/**
 * The pre-image of a received frame: its ingress header sum (vpcsum_hsum_t, include/vpcsum.h),
 * recorded by the GPU while it verifies the RX batch ({@link GpuCsumBatch#verifyFrames}), and the
 * rule that decides whether the egress flush may update the frame's L4 sum from it (VPCsum.F_PRE,
 * a VPCsum.PRE_HSUM entry) instead of summing the whole segment as getRawPacket(0) would
 * (AbstractPacket.java:15-22).
 *
 * The record sums every word of the L4 sum that an in-place setter can change: the pseudo-header
 * addresses (Ipv4Packet / Ipv6Packet.setSrc / setDst) and the L4 header -- ports, sequence and
 * acknowledgement numbers, flags, window, options (TcpPacket.java:31-100, TcpOption.setData
 * :561-569, UdpPacket.java:188-209).  So the update is Java's full recompute whatever those setters
 * wrote -- SwitchUtils.applyNat, buildSyn(Ack)PacketForProxyProtocol, checkAndUpdateMss's in-place
 * clamp -- provided that (1) the stored sum was correct on receipt (S_L4_OK) and (2) every other byte
 * of the segment and its length are the received ones.  (2) holds exactly while the frame leaves
 * from XDPIface.sendPacket's zero-copy branch with its L3 header where it was received: every other
 * change rebuilds the packet (clearRawPacket, e.g. TcpPacket.setData / setOptions, the MSS option
 * added by checkAndUpdateMss), which clears the PacketBuffer's buffers up the parent chain
 * (AbstractPacket.java:27-36, PacketBuffer.java:199-208), and PacketBuffer.replacePacket (TcpReset,
 * TcpStack, the ICMP answers) does the same and resets the fields below.  The GPU checks the lengths
 * once more and refuses (S_BAD_DESC, nothing written) a record that does not match.
 *
 * PacketBuffer gets three fields (INTEGRATION.md §5): {@code int csumStatus = -1} (the verify
 * status byte), {@code long csumHsum} (the 8-B record, 0 = none) and {@code long csumL3 = -1} (the L3
 * header's umem offset at receipt).  Not compiled in this repository (the build image has no JDK).
 */
public final class PreImage {
    private PreImage() {
    }

    /** The record's fields (little-endian vpcsum_hsum_t read as one long). */
    static int sum(long r) { return (int) (r & 0xffff); }
    static int l4Len(long r) { return (int) ((r >>> 16) & 0xffff); }
    static int hlen(long r) { return (int) ((r >>> 32) & 0xff); }
    static int proto(long r) { return (int) ((r >>> 40) & 0xff); }
    static int ver(long r) { return (int) ((r >>> 48) & 0xff); }
    static int l2Len(long r) { return (int) ((r >>> 56) & 0xff); }

    /**
     * XDPIface.readable, after the batch's verify: frame {@code i} of the batch, received at umem
     * offset {@code frameOff}, gets its status byte and record.
     */
    public static void received(PacketBuffer pkb, MemorySegment status, MemorySegment hsum, int i, long frameOff) {
        pkb.csumStatus = status.get(ValueLayout.JAVA_BYTE, i) & 0xff;
        long r = hsum.getAtIndex(ValueLayout.JAVA_LONG_UNALIGNED, i);
        pkb.csumHsum = r;
        pkb.csumL3 = l2Len(r) != 0 ? frameOff + l2Len(r) : -1;
    }

    /** PacketBuffer.clearPackets (every replacePacket / clearAndSetPacket): a new packet has no
     * verify status and no record. */
    public static void clear(PacketBuffer pkb) {
        pkb.csumStatus = -1;
        pkb.csumHsum = 0;
        pkb.csumL3 = -1;
    }

    /**
     * GpuCsumBatch.defer's rule: may the frame of {@code pkb}, leaving in {@code chunk} with its
     * L3 header at umem offset {@code l3} (version, protocol, lengths as the IP packet reports
     * them), take its L4 sum from its record?  {@code umem} is read for the TCP data offset now in
     * the frame (a partially parsed TcpPacket has no getDataOffset(), TcpPacket.java:186-199).
     */
    static boolean eligible(PacketBuffer pkb, ChunkInfo chunk, MemorySegment umem, long l3, int ver, int proto,
                            int l3len, int l4off) {
        long r = pkb.csumHsum;
        if (r == 0 || l2Len(r) == 0 || pkb.csumStatus < 0
            || (pkb.csumStatus & (VPCsum.S_L4_OK | VPCsum.S_BAD_DESC)) != VPCsum.S_L4_OK) {
            return false;
        }
        // the zero-copy branch of XDPIface.sendPacket: the PacketBuffer still holds the received
        // chunk (any rebuild or replacement nulled pkb.fullbuf), the L3 header where it was received
        if (!(pkb.fullbuf instanceof UMemChunkByteArray ub) || ub.chunk != chunk || l3 != pkb.csumL3) {
            return false;
        }
        if (ver(r) != ver || proto(r) != proto || l4Len(r) != l3len - l4off) {
            return false;
        }
        if (proto == 6) {
            int doff = ((umem.get(ValueLayout.JAVA_BYTE, l3 + l4off + 12) & 0xff) >>> 4) * 4;
            return hlen(r) == doff;
        }
        return proto == 17 && hlen(r) == 8;
    }

    /** The 48-B vpcsum_pre_t at {@code off} of {@code seg}: the record in its first 8 bytes, mask
     * PRE_HSUM at byte 36, the rest 0. */
    static void writeTo(MemorySegment seg, long off, long hsum) {
        seg.asSlice(off, VPCsum.PRE_ENTRY).fill((byte) 0);
        seg.set(ValueLayout.JAVA_LONG_UNALIGNED, off, hsum);
        seg.set(ValueLayout.JAVA_BYTE, off + 36, (byte) VPCsum.PRE_HSUM);
    }
}
