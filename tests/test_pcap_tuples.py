"""Flow tuples pinned on the reference's own table.

TestPcap.java lists, frame by frame, what vproxy's parsers must read from its three pcap fixtures:
src / dst address and port of the 27 TCP frames of cap-ether.pcap and cap-linux-cooked.pcap
(PktCheck lists, TestPcap.java:45-89, with the TCP flags each PktCheck declares) and the address
pairs of the 4 ICMP frames of cap-bsd-loopback-encap.pcap (:92-108).  tests/golden/make_golden.py
extracts the table into tests/golden/pcap_tuples.json (data).

The linux-cooked and BSD-loopback payloads are IP packets without an Ethernet header; they are put
behind one (EtherType from the IP version), as the vswitch would hold them, so the same Ethernet
parser (oracle.flow_tuple on the CPU, vpcsum_parse_ether_tuples_async on the GPU) reads them all.
"""
import ipaddress
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from pcaputil import l3_offset, read_pcap

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _frames_and_table():
    table = json.load(open(os.path.join(GOLD, "pcap_tuples.json")))["pcaps"]
    frames, rows = [], []
    for fn, spec in table.items():
        lt, pkts = read_pcap(os.path.join(GOLD, "pcap", fn))
        assert len(pkts) == len(spec["frames"]), fn
        for p, row in zip(pkts, spec["frames"]):
            o = l3_offset(lt, p)
            assert o is not None
            ip = p[o:]
            frames.append(p if o in (14, 18) and lt == 1 else
                          bytes(12) + (b"\x08\x00" if ip[0] >> 4 == 4 else b"\x86\xdd") + ip)
            rows.append(row)
    assert len(frames) == 31
    return frames, rows


def _want(row):
    """The tuple TestPcap expects, in vpcsum_tuple_t form (network-order bytes)."""
    def addr(s):
        b = ipaddress.ip_address(s).packed
        return b + bytes(16 - len(b))
    proto = row.get("proto", 6)
    sp = row.get("sport")
    dp = row.get("dport")
    return dict(src=addr(row["src"]), dst=addr(row["dst"]), l3_ver=4, l4_proto=proto,
                sport=None if sp is None else sp.to_bytes(2, "big"),
                dport=None if dp is None else dp.to_bytes(2, "big"),
                tcp_flags=row.get("tcp_flags"))


def test_oracle_tuples_equal_testpcap_table():
    """oracle.flow_tuple on all 31 frames equals TestPcap.java's expectations, TCP flags included."""
    frames, rows = _frames_and_table()
    for i, (f, row) in enumerate(zip(frames, rows)):
        t, w = O.flow_tuple(f), _want(row)
        assert (t["src"], t["dst"], t["l3_ver"], t["l4_proto"]) == (w["src"], w["dst"], 4, w["l4_proto"]), i
        if w["sport"] is not None:
            assert (t["sport"], t["dport"]) == (w["sport"], w["dport"]), i
            assert t["tcp_flags"] == w["tcp_flags"], (i, row)
        else:
            assert t["sport"] == bytes(2) and t["dport"] == bytes(2) and t["tcp_flags"] == 0


@pytest.mark.gpu
def test_gpu_tuples_equal_testpcap_table():
    """The GPU parser's tuples (vpcsum_parse_ether_tuples_async) on the same 31 frames equal the
    reference's table, at odd offsets in one arena."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vproxy_amd import vpcsum as V
    V.lib()
    frames, rows = _frames_and_table()
    offs, lens, arena = [], [], bytearray()
    for i, f in enumerate(frames):
        arena += bytes(1 + i % 3)
        offs.append(len(arena))
        lens.append(len(f))
        arena += f
    arena = np.frombuffer(bytes(arena) + bytes(64), np.uint8).copy()
    n = len(frames)
    ga = torch.from_numpy(arena).pin_memory().cuda()
    go = torch.from_numpy(np.array(offs, np.uint64)).pin_memory().cuda()
    gl = torch.from_numpy(np.array(lens, np.uint32)).pin_memory().cuda()
    d = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    tu = torch.full((n * V.TUPLE_DTYPE.itemsize,), 0xAB, dtype=torch.uint8, device="cuda")
    V.parse_ether(ga, go, gl, n, d, st, tuples=tu)
    torch.cuda.synchronize()
    got = tu.cpu().numpy().view(V.TUPLE_DTYPE)
    assert not (st.cpu().numpy() & V.S_BAD_DESC).any()
    for i, row in enumerate(rows):
        g, w = got[i], _want(row)
        assert (g["src"].tobytes(), g["dst"].tobytes(), int(g["l3_ver"]), int(g["l4_proto"])) == \
            (w["src"], w["dst"], 4, w["l4_proto"]), i
        if w["sport"] is not None:
            assert (g["sport"].tobytes(), g["dport"].tobytes(), int(g["tcp_flags"])) == \
                (w["sport"], w["dport"], w["tcp_flags"]), (i, row)
        else:
            assert g["sport"].tobytes() == bytes(2) and int(g["tcp_flags"]) == 0
