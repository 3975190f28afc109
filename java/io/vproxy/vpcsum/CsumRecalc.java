package io.vproxy.vpcsum;

import io.vproxy.vswitch.util.CSumRecalcType;

/**
 * The verify status of a received frame -> what DevInput.handle's csum-recalc step does with it
 * (core/src/main/java/io/vproxy/vswitch/node/DevInput.java:37-49, CSumRecalcType.java:3-6).
 * Same table as vproxy_amd/vswitch.py:recalc_policy and INTEGRATION.md §4.
 *
 * With {@code all} the reference clears every IP packet's sums, so egress recomputes all of them;
 * a sum that verified would be recomputed to the value it already holds, so only the failing
 * frames need the dirty mark for the frames to leave byte-identical.  A UDP stored 0 ("no
 * checksum") is marked too: Java's recompute replaces it with a real sum.
 *
 * Not compiled in this repository (no JDK in the build image).
 */
public final class CsumRecalc {
    /** clear the IP header checksum (ipPkt.clearChecksum()) */
    public static final int CLEAR_IP = 0x1;
    /** clear the upper-layer checksum (ipPkt.getPacket().clearChecksum()) */
    public static final int CLEAR_L4 = 0x2;
    /** drop the frame (opt-in, NIC-facing interfaces only) */
    public static final int DROP = 0x4;

    private CsumRecalc() {
    }

    /**
     * @param status  the frame's VPCsum.S_* byte from verifyFrames (negative: not verified)
     * @param hasIp   the frame has an IPv4 header sum (IPv4: the parse set F_IP)
     * @param hasL4   the frame's upper layer carries a sum (TCP / UDP / ICMP / ICMPv6)
     * @param type    the input interface's csum-recalc setting
     * @param dropBad drop frames whose stored sums fail instead of repairing them
     */
    public static int action(int status, boolean hasIp, boolean hasL4, CSumRecalcType type, boolean dropBad) {
        if (status < 0) { // no verify ran: today's behaviour
            if (type == CSumRecalcType.none) return 0;
            return CLEAR_L4 | (type == CSumRecalcType.all ? CLEAR_IP : 0);
        }
        if ((status & VPCsum.S_BAD_DESC) != 0) return 0; // PacketBytes to Java: untouched
        boolean ipBad = hasIp && (status & VPCsum.S_IP_OK) == 0;
        boolean l4Bad = hasL4 && (status & VPCsum.S_L4_OK) == 0;
        boolean noCsum = hasL4 && (status & VPCsum.S_UDP_NOCSUM) != 0;
        if (dropBad && (ipBad || (l4Bad && !noCsum))) return DROP;
        if (type != CSumRecalcType.all) return 0;
        return (ipBad ? CLEAR_IP : 0) | (l4Bad ? CLEAR_L4 : 0);
    }
}
