/*
 * vpcsum.h -- C-ABI of libvpcsum.so, the MI355X (gfx950) batched Internet
 * checksum engine for vproxy's vswitch.
 *
 * The library replaces the per-packet Java checksum path
 *   io.vproxy.base.util.Utils.calculateChecksum / calculateChecksumIntermediate /
 *   calculateChecksumDoFinal          (base/src/main/java/io/vproxy/base/util/Utils.java:778-801)
 *   Utils.buildPseudoIPv4Header / buildPseudoIPv6Header          (Utils.java:758-776)
 *   Ipv4Packet.__updateChecksum                                   (vpacket/Ipv4Packet.java:209-217)
 *   TcpPacket.updateChecksumWithIPv4 / IPv6                       (vpacket/TcpPacket.java:475-485, 508-518)
 *   UdpPacket.updateChecksumWithIPv4 / IPv6                       (vpacket/UdpPacket.java:136-164)
 *   IcmpPacket.__updateChecksum / updateChecksumWithIPv6          (vpacket/IcmpPacket.java:64-74, 124-135)
 * with ONE batched GPU launch per flush point (Iface.completeTx, Switch.java:1076-1078), in the
 * same flag-and-flush shape the XDP path already uses for its native checksum
 * (SwitchUtils.checksumFlagsFor, core/.../vswitch/util/SwitchUtils.java:297-316;
 *  XDPIface.sendPacket / completeTx, core/.../vswitch/iface/XDPIface.java:100-178, 227-243).
 *
 * Two entry-point families:
 *   1. vpcsum_*                      plain C, return 0 on success, <0 on error
 *                                    (message via vpcsum_last_error()).
 *   2. Java_io_vproxy_vpcsum_VPCsum_* PNI convention (base/src/main/c-generated/pni.h:15-82):
 *                                    int f(PNIEnv_<ret>* env, args...), 0 = ok, -1 = exception
 *                                    stored in env->ex, result in env->return_.
 *
 * No torch types, no CUDA types: plain pointers and sizes.  Device pointers are
 * hipMalloc'd (or torch) device memory; `stream` is a hipStream_t passed as void*.
 */
#ifndef VPCSUM_H
#define VPCSUM_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 4): VPCSUM_NAT_DEC_TTL refuses a TTL / hop limit <= 1 (S_BAD_DESC | S_TTL_EXPIRED)
 * instead of writing 0; vpcsum_synth_async takes a NULL arena (descriptors only).
 * 3 (round 5): VPCSUM_F_PRE and the pre-image entry points (vpcsum_pre_async,
 * vpcsum_ctx_submit_pre, vpcsum_group_submit_pre, vpcsum_batch_submit_pre, VPCsum.submitPre);
 * vpcsum_compute_async leaves F_PRE descriptors to vpcsum_pre_async; a handle of the process-wide
 * group from before a vpcsum_shutdown is refused.
 * 4 (round 6): the ingress header sum (vpcsum_hsum_t, VPCSUM_PRE_HSUM entries;
 * vpcsum_ctx_verify_frames_hsum, vpcsum_parse_ether_hsum_async, VPCsum.verifyFramesHsum): the
 * egress pre-image flush no longer depends on which setters ran; vpcsum_ctx_submit stages memory
 * the context has not registered instead of copying from it directly. */
#define VPCSUM_ABI_VERSION 4

/* ------------------------------------------------------------------------ */
/* Data formats                                                             */
/* ------------------------------------------------------------------------ */

/* Per-packet descriptor flags (which sums are dirty).
 * F_IP / F_L4 are the batched form of AbstractPacket.isRequireUpdatingChecksum()
 * on the IP packet and on its upper-layer packet (AbstractPacket.java:38-65,
 * Ipv4Packet.java:219-234, Ipv6Packet.java:219-236), i.e. XDP's VP_CSUM_IP / VP_CSUM_UP. */
#define VPCSUM_F_IP    0x01u /* IPv4 header checksum (field L3+10)                        */
#define VPCSUM_F_L4    0x02u /* TCP(+16) / UDP(+6) / ICMP(+2) / ICMPv6(+2) checksum        */
#define VPCSUM_F_L4P   0x08u /* checksum offload (VP_CSUM_UP_PSEUDO, SwitchUtils.java:297-316): the L4
                              * field gets the folded, uncomplemented pseudo-header sum, the value
                              * Linux stores for CHECKSUM_PARTIAL (the reference's pcap fixtures
                              * hold 12 such TCP frames); the device adds the segment sum.  Not
                              * with VPCSUM_F_L4; TCP / UDP / ICMPv6 only (ICMPv4 has no pseudo
                              * header).  VERIFY compares the stored field with that value.    */
#define VPCSUM_F_RAW   0x04u /* Utils.calculateChecksum(buf, len) over [l3_off, l3_off+l3_len);
                                result in out bits 0..15; nothing else is interpreted       */
#define VPCSUM_F_PRE   0x10u /* with VPCSUM_F_L4 and / or F_IP: the packet was NAT'd by Java's
                              * setters after its stored L4 sum was verified on ingress
                              * (VPCSUM_S_L4_OK); its L4 sum is updated by RFC 1624 from the
                              * packet's pre-image (vpcsum_pre_t: the words the setters
                              * overwrote, or with VPCSUM_PRE_HSUM the ingress header sum
                              * recorded on receipt) instead of summed over the segment, its IPv4 header
                              * sum recomputed.  Only the header is read.  Handled by
                              * vpcsum_pre_async / vpcsum_ctx_submit_pre; vpcsum_compute_async
                              * reads nothing of such a packet, writes nothing into its frame and
                              * reports out 0 / S_DONE for it.                                 */

typedef struct vpcsum_desc {
    uint64_t l3_off;   /* byte offset of the L3 (IP) header inside the arena               */
    uint16_t l3_len;   /* IPv4 totalLength / IPv6 40+payloadLength (L2 padding excluded,
                          Ipv4Packet.java:100-103, Ipv6Packet.java:103-106)                  */
    uint16_t l4_off;   /* L4 header offset relative to l3_off (ihl*4, or 40+ext headers)    */
    uint8_t  l3_ver;   /* 4 or 6                                                             */
    uint8_t  l4_proto; /* 6 TCP, 17 UDP, 1 ICMP, 58 ICMPv6; anything else: no L4 sum          */
    uint8_t  flags;    /* VPCSUM_F_*                                                          */
    uint8_t  rsv;      /* must be 0                                                          */
} vpcsum_desc_t;       /* 16 bytes, naturally aligned                                        */

/* Output word per packet: bits 0..15 = IPv4 header checksum, bits 16..31 = L4 checksum
 * (host-order values, exactly the ints Java writes with ByteArray.int16). */

/* Status byte per packet (optional output). */
#define VPCSUM_S_IP_OK       0x01u /* verify: stored IPv4 header checksum == recomputed   */
#define VPCSUM_S_L4_OK       0x02u /* verify: stored L4 checksum == recomputed            */
#define VPCSUM_S_UDP_NOCSUM  0x04u /* UDP with stored checksum 0 (RFC 768 "no checksum")  */
#define VPCSUM_S_TTL_EXPIRED 0x20u /* NAT: VPCSUM_NAT_DEC_TTL on a TTL / hop limit <= 1 (the value
                                    * after VPCSUM_NAT_SET_TTL when both are set): the packet is
                                    * refused with S_BAD_DESC and nothing is written.  The reference
                                    * never decrements such a packet: IPInputRoute drops it and
                                    * answers ICMP time exceeded (IPInputRoute.java:81-88)      */
#define VPCSUM_S_DONE        0x40u /* descriptor processed                                */
#define VPCSUM_S_BAD_DESC    0x80u /* descriptor rejected (bounds/lengths); nothing written */

/* Batch modes. */
#define VPCSUM_MODE_COMPUTE  0x00u /* compute dirty sums                                    */
#define VPCSUM_MODE_VERIFY   0x01u /* compute and compare with the stored fields (ingress)  */
#define VPCSUM_MODE_WRITE    0x10u /* also write results big-endian into the arena in place */

/* NAT / TTL rewrites (SwitchUtils.applyNat, core/.../vswitch/util/SwitchUtils.java:522-542): the
 * setters Ipv4Packet.setSrc/setDst (vpacket/Ipv4Packet.java:433-458), Ipv6Packet.setSrc/setDst
 * (Ipv6Packet.java:374-396), TcpPacket/UdpPacket.setSrcPort/setDstPort (TcpPacket.java:31-51,
 * UdpPacket.java:188-209), Ipv4Packet.setTtl (:401-407; IPInputRoute.java:79-91 decrements) and
 * Ipv6Packet.setHopLimit (:354-359), each followed by Java's recompute of the sums it dirtied.
 * Address and port bytes in NETWORK byte order, exactly the bytes written into the packet. */
#define VPCSUM_NAT_SRC      0x01u /* source address (IPv4 bytes 12..15 / IPv6 8..23)             */
#define VPCSUM_NAT_DST      0x02u /* destination address (IPv4 16..19 / IPv6 24..39)              */
#define VPCSUM_NAT_SPORT    0x04u /* TCP / UDP source port                                        */
#define VPCSUM_NAT_DPORT    0x08u /* TCP / UDP destination port                                   */
#define VPCSUM_NAT_DEC_TTL  0x10u /* IPv4 TTL / IPv6 hop limit minus 1 (after SET_TTL if both); a
                                   * value <= 1 refuses the packet (VPCSUM_S_TTL_EXPIRED)        */
#define VPCSUM_NAT_SET_TTL  0x20u /* IPv4 TTL / IPv6 hop limit := the entry's ttl value           */

/* IPv4-only entry, 16 bytes (BASELINE config C5: 72 algorithmic bytes per packet).
 * rsv[0] carries the VPCSUM_NAT_SET_TTL value; an IPv6 descriptor is rejected (S_BAD_DESC). */
typedef struct vpcsum_nat4 {
    uint8_t  src[4];
    uint8_t  dst[4];
    uint8_t  sport[2];
    uint8_t  dport[2];
    uint8_t  mask;     /* VPCSUM_NAT_*  */
    uint8_t  rsv[3];   /* rsv[0]: TTL value for VPCSUM_NAT_SET_TTL, others 0 */
} vpcsum_nat4_t;

/* IPv4 and IPv6 entry, 48 bytes: an IPv4 packet uses src[0..3] / dst[0..3]. */
typedef struct vpcsum_nat {
    uint8_t  src[16];
    uint8_t  dst[16];
    uint8_t  sport[2];
    uint8_t  dport[2];
    uint8_t  mask;     /* VPCSUM_NAT_*                                  */
    uint8_t  ttl;      /* TTL / hop limit value for VPCSUM_NAT_SET_TTL    */
    uint8_t  rsv[10];  /* 0                                             */
} vpcsum_nat_t;

/* IPv4 record, 32 bytes: a packet's descriptor and its IPv4 entry side by side, so the rewrite
 * kernel reads one stream of 32 B per packet instead of two of 16 B (vpcsum_nat4r_async). */
typedef struct vpcsum_nat4_rec {
    vpcsum_desc_t desc;
    vpcsum_nat4_t rw;
} vpcsum_nat4_rec_t;

/* NAT modes. */
#define VPCSUM_NAT_RFC1624     0x00u /* incremental update (RFC 1624 eqn. 3); header bytes only */
#define VPCSUM_NAT_STRICT_JAVA 0x01u /* rewrite, then full recompute: identical to Java for ANY
                                        input, including invalid input checksums              */

/* Pre-image of a packet NAT'd by Java's own setters (VPCSUM_F_PRE): the OLD addresses and ports,
 * recorded just before SwitchUtils.applyNat ran the setters (SwitchUtils.java:531-542), in the
 * layout of the NAT entries: vpcsum_pre_t = vpcsum_nat_t (48 B; an IPv4 packet uses src[0..3] /
 * dst[0..3]) and vpcsum_pre4_t = vpcsum_nat4_t (16 B, IPv4 only).  mask: VPCSUM_NAT_SRC / DST /
 * SPORT / DPORT, the fields recorded (a field recorded but not changed adds nothing); the TTL
 * bits and values are ignored: the IPv4 header sum is recomputed in full from the header. */
typedef vpcsum_nat_t vpcsum_pre_t;
typedef vpcsum_nat4_t vpcsum_pre4_t;
#define VPCSUM_PRE_FMT_PRE4 0u   /* vpcsum_pre4_t entries */
#define VPCSUM_PRE_FMT_PRE  1u   /* vpcsum_pre_t entries  */

/* Ingress header sum of a received TCP / UDP frame, recorded by the RX verify
 * (vpcsum_ctx_verify_frames_hsum) from the frame as it arrived.  `sum` is the one's complement sum
 * (16-bit big-endian words, folded end-around; host order) of every word of the L4 sum that the
 * vswitch's in-place setters can reach: the pseudo-header addresses (IPv4 L3+12..19, IPv6
 * L3+8..39) and the L4 header's words [0, hlen) except the checksum field -- ports, sequence and
 * acknowledgement numbers, flags, window, options (TcpPacket.java:31-110, TcpOption.setData
 * :561-569; UdpPacket.java:188-209; Ipv4Packet/Ipv6Packet.setSrc/setDst).  At egress
 * (VPCSUM_PRE_HSUM) the L4 sum is updated from it, RFC 1624 eqn. 3 with the header as one word:
 * HC' = ~(~HC + ~sum + sum'), sum' the same words of the frame now.  That equals Java's full
 * recompute (getRawPacket(0), AbstractPacket.java:15-22) for ANY change of those words, provided the
 * stored HC was correct on receipt (VPCSUM_S_L4_OK) and the payload and lengths are the received
 * ones: the caller's part (INTEGRATION.md §5 gives the vswitch's rule).  l2_len = 0: no record
 * (not TCP / UDP, a refused frame, a segment shorter than its header). */
typedef struct vpcsum_hsum {
    uint16_t sum;
    uint16_t l4_len;   /* segment length on receipt: l3_len - l4_off                         */
    uint8_t  hlen;     /* L4 header bytes summed: TCP data offset * 4 (20..60), UDP 8         */
    uint8_t  l4_proto; /* 6 / 17                                                              */
    uint8_t  l3_ver;   /* 4 / 6                                                               */
    uint8_t  l2_len;   /* 14 / 18 (802.1Q): the L3 header's offset in the frame; 0: no record  */
} vpcsum_hsum_t;       /* 8 bytes */

/* vpcsum_pre_t / vpcsum_pre4_t mask bit: the entry's first 8 bytes (src[0..7], or src[0..3] and
 * dst[0..3] of a vpcsum_pre4_t) hold the packet's vpcsum_hsum_t instead of old addresses and
 * ports (the other mask bits are then ignored).  The packet is refused (S_BAD_DESC, nothing
 * written) unless its version, protocol, segment length and L4 header length (the TCP data offset
 * now in the frame) equal the record's. */
#define VPCSUM_PRE_HSUM 0x80u

/* ------------------------------------------------------------------------ */
/* Library / device                                                         */
/* ------------------------------------------------------------------------ */
int         vpcsum_abi_version(void);
const char* vpcsum_last_error(void);          /* thread-local message of the last failure */
int         vpcsum_device_count(int* out_n);
int         vpcsum_set_device(int device);

/* ------------------------------------------------------------------------ */
/* Device-resident batch ops (async on `stream`; all pointers device memory) */
/* ------------------------------------------------------------------------ */

/* Compute / verify the checksums named by each descriptor's flags.
 * d_out (n words) and d_status (n bytes) may each be NULL. */
int vpcsum_compute_async(const uint8_t* d_arena, uint64_t arena_len,
                         const vpcsum_desc_t* d_desc, uint32_t n,
                         uint32_t* d_out, uint8_t* d_status,
                         uint32_t mode, void* stream);

/* Two batches in flight.  A launch spends its first and last microseconds
 * ramping up and draining; a caller that keeps two batches in flight overlaps those with its
 * neighbour's steady state (C1, 64-B frames: +29%).  A pipe owns two streams on the
 * caller's device: vpcsum_pipe_begin forks them from `stream` (they wait for the work queued on it
 * so far), each vpcsum_pipe_compute_async (vpcsum_compute_async's arguments) goes to the next of the
 * two in turn, so consecutive batches may run concurrently -- their out / status / written frames
 * must not overlap -- and vpcsum_pipe_join makes `stream` wait for every batch launched since.  The
 * host contexts do the same on their own: each keeps two slots, each with its stream, and a submit
 * goes to the other slot than the last (wait for ticket t before reusing t's buffers). */
typedef struct vpcsum_pipe vpcsum_pipe_t;
int vpcsum_pipe_create(void* stream, vpcsum_pipe_t** out);
int vpcsum_pipe_begin(vpcsum_pipe_t* pipe);
int vpcsum_pipe_compute_async(vpcsum_pipe_t* pipe, const uint8_t* d_arena, uint64_t arena_len,
                              const vpcsum_desc_t* d_desc, uint32_t n, uint32_t* d_out, uint8_t* d_status,
                              uint32_t mode);
int vpcsum_pipe_join(vpcsum_pipe_t* pipe);
int vpcsum_pipe_destroy(vpcsum_pipe_t* pipe);

/* NAT / TTL rewrite + checksum update, in place in the arena; d_rw[i] rewrites packet i.
 * d_status (n bytes): S_DONE, or S_BAD_DESC for a rejected descriptor (nothing written);
 * required with VPCSUM_NAT_STRICT_JAVA. */
int vpcsum_nat4_async(uint8_t* d_arena, uint64_t arena_len,
                      const vpcsum_desc_t* d_desc, const vpcsum_nat4_t* d_rw, uint32_t n,
                      uint8_t* d_status, uint32_t nat_mode, void* stream);
int vpcsum_nat_async(uint8_t* d_arena, uint64_t arena_len,
                     const vpcsum_desc_t* d_desc, const vpcsum_nat_t* d_rw, uint32_t n,
                     uint8_t* d_status, uint32_t nat_mode, void* stream);
/* vpcsum_nat4_async over records (descriptor + entry per packet, one read stream); IPv4 only,
 * VPCSUM_NAT_RFC1624 only (the strict-Java recompute reads plain descriptors). */
int vpcsum_nat4r_async(uint8_t* d_arena, uint64_t arena_len, const vpcsum_nat4_rec_t* d_rec, uint32_t n,
                       uint8_t* d_status, uint32_t nat_mode, void* stream);

/* Egress sums of NAT'd packets from their pre-images: every descriptor with VPCSUM_F_PRE gets its
 * L4 sum by RFC 1624 eqn. 3 from the stored field, the old words d_pre[i] records and the words now
 * in the frame (HC' = ~(~HC + sum(~m + m'))) -- with VPCSUM_PRE_HSUM, the recorded header sum and the
 * same header words now (any in-place change of them) --, its IPv4 header sum (F_IP) recomputed in full from the
 * header; a UDP stored 0 (no checksum) is summed in full.  The results equal Java's full recompute
 * (getRawPacket(0) after the setters, AbstractPacket.java:15-22) whenever the stored L4 sum was
 * correct before the rewrite -- what ingress verify's VPCSUM_S_L4_OK proves -- and nothing but the
 * recorded fields changed since.  pre_fmt: VPCSUM_PRE_FMT_PRE4 (IPv4 only) or VPCSUM_PRE_FMT_PRE.
 * mode: VPCSUM_MODE_WRITE to store the sums into the frames.  Out / status as vpcsum_compute_async
 * (S_BAD_DESC: F_PRE without F_L4 or F_IP, with F_L4P / F_RAW, F_IP on IPv6, an IPv6 packet with
 * 16-B entries, bounds).  d_pre holds n entries; those of descriptors without F_PRE are ignored.  Descriptors without F_PRE are not touched (out / status not written): run
 * vpcsum_compute_async on the same batch first, on the same stream, for them. */
int vpcsum_pre_async(uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc, const void* d_pre,
                     uint32_t pre_fmt, uint32_t n, uint32_t* d_out, uint8_t* d_status, uint32_t mode, void* stream);

/* Build descriptors on the GPU by parsing Ethernet frames (EthernetPacket.from,
 * Ipv4Packet.from, Ipv6Packet.from rules). frame i = [d_frame_off[i], +d_frame_len[i]).
 * flags = VPCSUM_F_* applied to every IP packet found; non-IP / unparsable frames get
 * flags 0 and status VPCSUM_S_BAD_DESC. */
int vpcsum_parse_ether_async(const uint8_t* d_arena, uint64_t arena_len,
                             const uint64_t* d_frame_off, const uint32_t* d_frame_len, uint32_t n,
                             uint8_t flags, vpcsum_desc_t* d_desc, uint8_t* d_status, void* stream);

/* Flow tuple of a parsed frame: what the vswitch's L4 input nodes read before their conntrack
 * lookup (TcpInput.java:47-51: tcpPkt.getSrc(ipPkt) / getDst(ipPkt) -> conntrack.lookupTcp, and
 * getFlags() == SYN -> lookupTcpListen; UdpInput.java:45-47: IPPort(ipPkt.getDst(),
 * udpPkt.getDstPort()) -> lookupUdpListen), and what SwitchUtils.executeTcpNat / executeUdpNat
 * compare (:321-322, :506-507).  Addresses and ports in network order; an IPv4 address is the
 * first 4 bytes (zeros after).  Ports (TcpPacket / UdpPacket.initPartial: uint16 at 0 and 2) and
 * tcp_flags (TcpPacket.initPartial :192-195: uint16 at 12 & 0x3f) are 0 for other protocols.  A
 * refused frame (status S_BAD_DESC) gets an all-zero tuple (l3_ver 0). */
typedef struct vpcsum_tuple {
    uint8_t src[16];
    uint8_t dst[16];
    uint8_t sport[2];
    uint8_t dport[2];
    uint8_t l3_ver;      /* 4 / 6; 0: refused frame */
    uint8_t l4_proto;
    uint8_t tcp_flags;
    uint8_t rsv;
} vpcsum_tuple_t;        /* 40 bytes */

/* vpcsum_parse_ether_async that also writes one vpcsum_tuple_t per frame to d_tuples (batched
 * header parse + tuple extraction), in the same pass over the headers. */
int vpcsum_parse_ether_tuples_async(const uint8_t* d_arena, uint64_t arena_len,
                                    const uint64_t* d_frame_off, const uint32_t* d_frame_len, uint32_t n,
                                    uint8_t flags, vpcsum_desc_t* d_desc, uint8_t* d_status,
                                    vpcsum_tuple_t* d_tuples, void* stream);

/* vpcsum_parse_ether_async that also writes each frame's ingress header sum (vpcsum_hsum_t,
 * l2_len 0 for a frame without one) to d_hsum, from the header bytes the parse reads. */
int vpcsum_parse_ether_hsum_async(const uint8_t* d_arena, uint64_t arena_len,
                                  const uint64_t* d_frame_off, const uint32_t* d_frame_len, uint32_t n,
                                  uint8_t flags, vpcsum_desc_t* d_desc, uint8_t* d_status,
                                  vpcsum_hsum_t* d_hsum, void* stream);

/* Streaming-read ceiling probe: reads `bytes` from d_buf with 16-B lanes, writes one word per
 * block into d_sink.  Used by bench.py to report a measured HBM read roof next to 8 TB/s. */
int vpcsum_read_probe_async(const uint8_t* d_buf, uint64_t bytes, uint32_t* d_sink,
                            uint32_t grid, void* stream);

/* Pattern read ceiling: reads exactly the 16-B chunks the checksum kernel reads for each
 * descriptor's L3 range (teams of 8 lanes, non-temporal), with no checksum work, and writes
 * one word per block into d_sink[0..1023].  grid 0 = 8 blocks per CU; grid bit 31 set = walk the
 * packets in the checksum kernel's unit order instead of grid-consecutively.  Arenas < 4 GiB.
 * Tooling: prices a workload's frame layout. */
int vpcsum_pattern_probe_async(const uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc,
                               uint32_t n, uint32_t* d_sink, uint32_t grid, void* stream);

/* NAT pattern ceiling: the memory operations of vpcsum_nat4_async (RFC 1624, wide kernel) for a
 * rewrite of both addresses and both ports -- descriptor and entry reads, the header window loads,
 * the one contiguous store of [L3+10, end of the L4 checksum field) -- with no rewrite: every byte
 * is stored back unchanged.  Tooling: prices BASELINE config C5's access pattern. */
int vpcsum_nat4_pattern_probe_async(uint8_t* d_arena, uint64_t arena_len, const vpcsum_desc_t* d_desc,
                                    const vpcsum_nat4_t* d_rw, uint32_t n, void* stream);
/* The same over records (vpcsum_nat4r_async's memory operations with no rewrite). */
int vpcsum_nat4r_pattern_probe_async(uint8_t* d_arena, uint64_t arena_len, const vpcsum_nat4_rec_t* d_rec,
                                     uint32_t n, void* stream);

/* Synthetic workload generator (bench / tests): deterministic counter-based splitmix64 bytes,
 * identical to oracle/csum_oracle.c:orc_synth_frame.  workload: see VPCSUM_SYNTH_*.  d_arena NULL
 * (with d_desc set): the descriptors alone, e.g. the lengths a rank needs to cut one global batch
 * into byte-balanced shards before it generates only its own. */
#define VPCSUM_SYNTH_C1_UDP64     1  /* IPv4/UDP L3 50 B                     */
#define VPCSUM_SYNTH_C2_TCP1500   2  /* IPv4/TCP L3 1500 B                   */
#define VPCSUM_SYNTH_C3_MIXED     3  /* IPv4 {64,576,1500} x {UDP,TCP,ICMP}  */
#define VPCSUM_SYNTH_C4_V6JUMBO   4  /* IPv6/TCP L3 9000 B                   */
#define VPCSUM_SYNTH_FUZZ         5  /* v4/v6, options, odd lengths, all protos */
#define VPCSUM_SYNTH_C5_NAT1500   6  /* IPv4 L3 1500 B, TCP or UDP (50/50): NAT input */
int vpcsum_synth_async(uint8_t* d_arena, uint64_t arena_len, uint32_t n, uint32_t stride,
                       uint32_t l3_pad, uint32_t workload, uint64_t seed, uint64_t first_index,
                       vpcsum_desc_t* d_desc, void* stream);

/* Tooling: a grid of `workgroups` x `threads` (a multiple of 64) that stays resident for `micros`
 * doing nothing but s_sleep -- no memory traffic.  The control of the A/B that asks whether a
 * resident kernel on another queue, as such, slows launched batches. */
int vpcsum_spin_probe_async(uint32_t workgroups, uint32_t threads, uint32_t micros, void* stream);

/* Kernel timing on the caller's stream (HIP events). */
int vpcsum_event_create(void** ev);
int vpcsum_event_destroy(void* ev);
int vpcsum_event_record(void* ev, void* stream);
int vpcsum_event_elapsed_ms(void* start, void* end, float* ms);
int vpcsum_stream_sync(void* stream);

/* ------------------------------------------------------------------------ */
/* Host-memory API (what the Java side drives): host arena + descriptors,   */
/* library-owned device buffers, pinned staging, async submit / wait.        */
/* ------------------------------------------------------------------------ */
typedef struct vpcsum_ctx vpcsum_ctx_t;

int vpcsum_ctx_create(int device, uint64_t max_arena_bytes, uint32_t max_pkts, vpcsum_ctx_t** out);
int vpcsum_ctx_destroy(vpcsum_ctx_t* ctx);
/* Page-lock a long-lived host arena (e.g. an AF_XDP umem, UMem.java:36-44) once, so that
 * submits from it DMA directly without a staging copy. */
int vpcsum_ctx_register_arena(vpcsum_ctx_t* ctx, void* h_arena, uint64_t len);
int vpcsum_ctx_unregister_arena(vpcsum_ctx_t* ctx, void* h_arena);
/* Copy the frames the descriptors touch to the device, run the batch, copy results back
 * (and, with VPCSUM_MODE_WRITE, the checksum fields back into the host frames).
 * Returns a ticket; results are valid after vpcsum_ctx_wait(ticket). */
int vpcsum_ctx_submit(vpcsum_ctx_t* ctx, uint8_t* h_arena, uint64_t arena_len,
                      const vpcsum_desc_t* h_desc, uint32_t n,
                      uint32_t* h_out, uint8_t* h_status, uint32_t mode, uint64_t* ticket);
int vpcsum_ctx_wait(vpcsum_ctx_t* ctx, uint64_t ticket);
/* Low-latency flushes (idle_us > 0): zero-copy batches of up to 512 frames from a registered arena
 * -- vpcsum_ctx_submit, vpcsum_ctx_submit_pre, vpcsum_ctx_egress_frames, vpcsum_ctx_verify_frames,
 * vpcsum_ctx_parse_frames -- are handed to a small persistent grid that polls a pinned mailbox,
 * instead of a kernel launch + event wait per batch (the Iface.completeTx flush of a few dozen
 * frames, XDPIface.java:227-243, and the RX poll).  Batches then run one at a time.  The grid leaves
 * after idle_us without a batch and is restarted by the next one; an idle grid costs launched batches
 * beside it nothing measurable (its pollers use relaxed loads), so larger batches,
 * which are launched, leave it resident.  idle_us = 0 stops it (the default).  Staged submits are
 * unaffected. */
int vpcsum_ctx_set_service(vpcsum_ctx_t* ctx, uint32_t idle_us);
/* Counters of a context: batches the service ran, service grids launched (either may be NULL). */
int vpcsum_ctx_stats(vpcsum_ctx_t* ctx, uint64_t* service_batches, uint64_t* service_launches);
/* Ingress verify of a received batch (XDPIface.readable, XDPIface.java:281-314): the raw Ethernet
 * frames at h_frame_off[i] (h_frame_len[i] bytes) of a registered arena are parsed on the GPU with
 * the rules of EthernetPacket/Ipv4Packet/Ipv6Packet.from (as vpcsum_parse_ether_async) and
 * verified (VPCSUM_MODE_VERIFY) where they lie, in one submission.  h_status[i]: S_DONE |
 * S_IP_OK | S_L4_OK | S_UDP_NOCSUM, or S_BAD_DESC for a frame that does not parse; h_out (may
 * be NULL): the sums the frames should carry.  Returns a ticket for vpcsum_ctx_wait. */
int vpcsum_ctx_verify_frames(vpcsum_ctx_t* ctx, const uint8_t* h_arena, uint64_t arena_len,
                             const uint64_t* h_frame_off, const uint32_t* h_frame_len, uint32_t n,
                             uint32_t* h_out, uint8_t* h_status, uint64_t* ticket);
/* vpcsum_ctx_verify_frames that also records every frame's ingress header sum in h_hsum (n
 * vpcsum_hsum_t, valid at vpcsum_ctx_wait): what the egress flush of the frame needs for a
 * VPCSUM_PRE_HSUM pre-image after the vswitch's in-place setters ran. */
int vpcsum_ctx_verify_frames_hsum(vpcsum_ctx_t* ctx, const uint8_t* h_arena, uint64_t arena_len,
                                  const uint64_t* h_frame_off, const uint32_t* h_frame_len, uint32_t n,
                                  uint32_t* h_out, uint8_t* h_status, vpcsum_hsum_t* h_hsum, uint64_t* ticket);
/* Batched parse of a received batch with flow tuples (the conntrack key TcpInput / UdpInput read,
 * TcpInput.java:47-51, UdpInput.java:45-47): the frames of a registered arena, as for
 * vpcsum_ctx_verify_frames, are parsed on the GPU where they lie; at vpcsum_ctx_wait h_desc[i]
 * holds frame i's descriptor (l3_off relative to h_arena, flags F_IP | F_L4 as the frame allows),
 * h_status[i] 0 or S_BAD_DESC, h_tuples[i] its vpcsum_tuple_t (any of the three may be NULL).
 * The descriptors can go straight to vpcsum_ctx_submit / vpcsum_ctx_nat_submit. */
int vpcsum_ctx_parse_frames(vpcsum_ctx_t* ctx, const uint8_t* h_arena, uint64_t arena_len,
                            const uint64_t* h_frame_off, const uint32_t* h_frame_len, uint32_t n,
                            vpcsum_desc_t* h_desc, uint8_t* h_status, vpcsum_tuple_t* h_tuples,
                            uint64_t* ticket);
/* Egress flush straight from the frames (the alternative to building descriptors on the host): the
 * frames at h_frame_off[i] (h_frame_len[i] bytes) of a registered arena, as the TX ring sends them
 * (XDPIface.sendPacket: chunk.getAddr() + pkb.pktOff and pkb.pktBuf.length(), or the copy's
 * pktaddr), each with the VPCSUM_F_* sums it needs (h_frame_flags[i]: F_IP / F_L4 / F_L4P, the
 * mapping of SwitchUtils.checksumFlagsFor, SwitchUtils.java:297-316).  The GPU parses every frame
 * with the vswitch's rules (as vpcsum_parse_ether_async: L3 after the Ethernet / 802.1Q header,
 * lengths from totalLength / payloadLength, L4 after IHL / the extension header), so padding,
 * options and extension headers are placed as Java's recompute places them, and writes the sums
 * into the frames (MODE_WRITE), in one submission.  At vpcsum_ctx_wait h_status[i] is S_DONE, or
 * S_BAD_DESC (nothing written) for a frame the parser refuses or whose flags it cannot honour (an
 * IPv4 header sum on IPv6, an L4 sum its segment cannot hold, F_L4P for ICMPv4): hand such a frame
 * back to the native path.  h_out (may be NULL): the sums, as vpcsum_ctx_submit. */
int vpcsum_ctx_egress_frames(vpcsum_ctx_t* ctx, uint8_t* h_arena, uint64_t arena_len,
                             const uint64_t* h_frame_off, const uint32_t* h_frame_len,
                             const uint8_t* h_frame_flags, uint32_t n,
                             uint32_t* h_out, uint8_t* h_status, uint64_t* ticket);
/* NAT / TTL rewrites of host frames (SwitchUtils.applyNat for a batch): h_rw[i] rewrites the
 * packet of h_desc[i] in place in the caller's frames, with the checksums updated as Java's
 * recompute leaves them (nat_mode as vpcsum_nat_async).  Frames in a registered arena are
 * rewritten where they lie (zero-copy); others are staged to the device and their rewritten
 * header bytes (L3 header through the L4 checksum field) copied back at vpcsum_ctx_wait.
 * h_status (may be NULL): S_DONE / S_BAD_DESC per packet.  Frames of one batch must not overlap. */
int vpcsum_ctx_nat_submit(vpcsum_ctx_t* ctx, uint8_t* h_arena, uint64_t arena_len,
                          const vpcsum_desc_t* h_desc, const vpcsum_nat_t* h_rw, uint32_t n,
                          uint8_t* h_status, uint32_t nat_mode, uint64_t* ticket);
/* The egress flush of a batch holding NAT'd frames: vpcsum_ctx_submit where
 * descriptors with VPCSUM_F_PRE take their L4 sum from h_pre[i] (pre_fmt as vpcsum_pre_async;
 * entries of other descriptors are ignored) and the others are summed in full, in one submission.
 * Frames of a registered arena are read and written in place (an F_PRE packet: its header only);
 * others are staged, an F_PRE packet's header only (its whole segment when it is UDP with a stored
 * 0).  mode: VPCSUM_MODE_COMPUTE / VPCSUM_MODE_WRITE (not VERIFY).  A batch of up to 512 packets
 * from a registered arena goes to the low-latency service grid when it is on
 * (vpcsum_ctx_set_service), F_PRE frames and the others together; larger ones are launched.  The
 * entries' rsv bytes are ignored. */
int vpcsum_ctx_submit_pre(vpcsum_ctx_t* ctx, uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc,
                          const void* h_pre, uint32_t pre_fmt, uint32_t n, uint32_t* h_out, uint8_t* h_status,
                          uint32_t mode, uint64_t* ticket);
/* Pipelined host->device->host throughput helper: processes a host arena of n fixed-stride
 * frames in `chunks` double-buffered pieces over two streams (H2D || kernel || D2H).  The arena,
 * descriptors and h_out must be registered (page-locked); with VPCSUM_MODE_WRITE the checksum
 * fields are also stored into the host frames (through the arena's mapping). */
int vpcsum_ctx_pipeline(vpcsum_ctx_t* ctx, uint8_t* h_arena, uint32_t stride, uint32_t copy_bytes,
                        const vpcsum_desc_t* h_desc, uint32_t n, uint32_t* h_out,
                        uint32_t mode, uint32_t chunks);

/* ------------------------------------------------------------------------ */
/* Device groups (multi-GPU host batches): one context per GPU in dev_mask;  */
/* a submitted batch is cut into contiguous descriptor ranges of nearly      */
/* equal byte totals (prefix sum of l3_len), one per GPU, each processed by  */
/* its own context; wait joins them.  No data crosses devices.               */
/* ------------------------------------------------------------------------ */
typedef struct vpcsum_group vpcsum_group_t;
int vpcsum_group_create(uint64_t dev_mask, uint64_t max_arena_bytes, uint32_t max_pkts, vpcsum_group_t** out);
/* devices[0..ndev): a device may repeat (several contexts on one GPU) */
int vpcsum_group_create_list(const int* devices, int ndev, uint64_t max_arena_bytes, uint32_t max_pkts,
                             vpcsum_group_t** out);
int vpcsum_group_destroy(vpcsum_group_t* g);
/* page-lock once (portable: every GPU of the group maps it) */
int vpcsum_group_register_arena(vpcsum_group_t* g, void* h_arena, uint64_t len);
/* finish every zero-copy batch still reading the arena on each device, then unpin it */
int vpcsum_group_unregister_arena(vpcsum_group_t* g, void* h_arena);
/* as vpcsum_ctx_submit, capacity per GPU; h_out / h_status hold all n results in batch order */
int vpcsum_group_submit(vpcsum_group_t* g, uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc,
                        uint32_t n, uint32_t* h_out, uint8_t* h_status, uint32_t mode, uint64_t* ticket);
int vpcsum_group_wait(vpcsum_group_t* g, uint64_t ticket);
/* as vpcsum_ctx_nat_submit, cut over the group's devices like vpcsum_group_submit; h_rw[i]
 * rewrites the packet of h_desc[i]; the ticket is joined by vpcsum_group_wait */
int vpcsum_group_nat_submit(vpcsum_group_t* g, uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc,
                            const vpcsum_nat_t* h_rw, uint32_t n, uint8_t* h_status, uint32_t nat_mode,
                            uint64_t* ticket);
/* as vpcsum_ctx_submit_pre, cut over the group's devices like vpcsum_group_submit */
int vpcsum_group_submit_pre(vpcsum_group_t* g, uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc,
                            const void* h_pre, uint32_t pre_fmt, uint32_t n, uint32_t* h_out, uint8_t* h_status,
                            uint32_t mode, uint64_t* ticket);

/* ------------------------------------------------------------------------ */
/* SURVEY.md §8(b)'s entry points: the same over ONE process-wide group.     */
/* vpcsum_init(dev_mask) creates it (error if one exists), vpcsum_shutdown   */
/* destroys it; the others fail with "vpcsum_init first" before it.  The     */
/* handle of a submit is waited on with vpcsum_batch_wait (checksum and NAT  */
/* batches alike).  vpcsum_shutdown first completes every batch still in     */
/* flight (results delivered into the callers' buffers); a handle issued     */
/* before it is then refused by vpcsum_batch_wait ("before vpcsum_shutdown"),*/
/* also after a new vpcsum_init.                                             */
/* ------------------------------------------------------------------------ */
int vpcsum_init(uint64_t dev_mask, uint64_t max_arena_bytes, uint32_t max_pkts);
int vpcsum_shutdown(void);
int vpcsum_register_arena(void* h_arena, uint64_t len);
int vpcsum_batch_submit(uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc, uint32_t n,
                        uint32_t* h_out, uint8_t* h_status, uint32_t mode, uint64_t* handle);
int vpcsum_batch_submit_pre(uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc, const void* h_pre,
                            uint32_t pre_fmt, uint32_t n, uint32_t* h_out, uint8_t* h_status, uint32_t mode,
                            uint64_t* handle);
int vpcsum_nat_submit(uint8_t* h_arena, uint64_t arena_len, const vpcsum_desc_t* h_desc, const vpcsum_nat_t* h_rw,
                      uint32_t n, uint8_t* h_status, uint32_t nat_mode, uint64_t* handle);
int vpcsum_batch_wait(uint64_t handle);

/* ------------------------------------------------------------------------ */
/* PNI entry points (bound by io.vproxy.vpcsum.VPCsum)   */
/* Layout copied from the PNI convention, base/src/main/c-generated/pni.h   */
/* ------------------------------------------------------------------------ */
typedef struct PNIException_vpcsum {
    char*   type;
    char    message[4096];
    int32_t errno_;    /* EINVAL (IllegalArgumentException) / EIO (IOException) on a throw */
} PNIException_vpcsum;   /* sizeof 4112: message at 8, errno_ at 4104 (tests/cpp/pni_layout.c) */

typedef struct PNIEnv_vpcsum_long {
    PNIException_vpcsum ex;
    union { int64_t return_; struct { uint64_t a, b; } placeholder_; };
} PNIEnv_vpcsum_long;   /* sizeof 4128, return_ at 4112: PNIEnv_long of pni.h */

typedef struct PNIEnv_vpcsum_int {
    PNIException_vpcsum ex;
    union { int32_t return_; struct { uint64_t a, b; } placeholder_; };
} PNIEnv_vpcsum_int;

typedef struct PNIEnv_vpcsum_void {
    PNIException_vpcsum ex;
    struct { uint64_t a, b; } placeholder_;
} PNIEnv_vpcsum_void;

/* VPCsum.create(int device, long maxArena, int maxPkts) -> long ctx */
int Java_io_vproxy_vpcsum_VPCsum_create(PNIEnv_vpcsum_long* env, int32_t device, int64_t maxArena, int32_t maxPkts);
/* VPCsum.registerArena(long ctx, MemorySegment arena, long len) */
int Java_io_vproxy_vpcsum_VPCsum_registerArena(PNIEnv_vpcsum_void* env, int64_t ctx, void* arena, int64_t len);
/* VPCsum.submit(long ctx, MemorySegment arena, long arenaLen, MemorySegment desc, int n,
 *               MemorySegment out, MemorySegment status, int mode) -> long ticket */
int Java_io_vproxy_vpcsum_VPCsum_submit(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                        void* desc, int32_t n, void* out, void* status, int32_t mode);
/* VPCsum.verifyFrames(long ctx, MemorySegment arena, long arenaLen, MemorySegment frameOff,
 *                     MemorySegment frameLen, int n, MemorySegment out, MemorySegment status) -> long ticket */
int Java_io_vproxy_vpcsum_VPCsum_verifyFrames(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                              void* frameOff, void* frameLen, int32_t n, void* out, void* status);
/* VPCsum.verifyFramesHsum(long ctx, MemorySegment arena, long arenaLen, MemorySegment frameOff,
 *                         MemorySegment frameLen, int n, MemorySegment out, MemorySegment status,
 *                         MemorySegment hsum) -> long ticket (vpcsum_ctx_verify_frames_hsum) */
int Java_io_vproxy_vpcsum_VPCsum_verifyFramesHsum(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                                  void* frameOff, void* frameLen, int32_t n, void* out, void* status,
                                                  void* hsum);
/* VPCsum.parseFrames(long ctx, MemorySegment arena, long arenaLen, MemorySegment frameOff,
 *                    MemorySegment frameLen, int n, MemorySegment desc, MemorySegment status,
 *                    MemorySegment tuples) -> long ticket */
int Java_io_vproxy_vpcsum_VPCsum_parseFrames(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                             void* frameOff, void* frameLen, int32_t n, void* desc, void* status,
                                             void* tuples);
/* VPCsum.egressFrames(long ctx, MemorySegment arena, long arenaLen, MemorySegment frameOff,
 *                     MemorySegment frameLen, MemorySegment frameFlags, int n, MemorySegment out,
 *                     MemorySegment status) -> long ticket */
int Java_io_vproxy_vpcsum_VPCsum_egressFrames(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                              void* frameOff, void* frameLen, void* frameFlags, int32_t n, void* out,
                                              void* status);
/* VPCsum.submitPre(long ctx, MemorySegment arena, long arenaLen, MemorySegment desc,
 *                  MemorySegment pre, int n, MemorySegment out, MemorySegment status, int mode)
 *   -> long ticket (vpcsum_ctx_submit_pre with 48-B vpcsum_pre_t entries) */
int Java_io_vproxy_vpcsum_VPCsum_submitPre(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                           void* desc, void* pre, int32_t n, void* out, void* status, int32_t mode);
/* VPCsum.natSubmit(long ctx, MemorySegment arena, long arenaLen, MemorySegment desc,
 *                  MemorySegment rw, int n, MemorySegment status, int natMode) -> long ticket */
int Java_io_vproxy_vpcsum_VPCsum_natSubmit(PNIEnv_vpcsum_long* env, int64_t ctx, void* arena, int64_t arenaLen,
                                           void* desc, void* rw, int32_t n, void* status, int32_t natMode);
/* VPCsum.setService(long ctx, int idleUs) */
int Java_io_vproxy_vpcsum_VPCsum_setService(PNIEnv_vpcsum_void* env, int64_t ctx, int32_t idleUs);
/* VPCsum.waitFor(long ctx, long ticket) */
int Java_io_vproxy_vpcsum_VPCsum_waitFor(PNIEnv_vpcsum_void* env, int64_t ctx, int64_t ticket);
/* VPCsum.close(long ctx) */
int Java_io_vproxy_vpcsum_VPCsum_close(PNIEnv_vpcsum_void* env, int64_t ctx);

#ifdef __cplusplus
}
#endif
#endif /* VPCSUM_H */
