"""Generate tests/golden/ fixtures from the reference's own test data (run in the build
container only; /root/reference does not exist on the GPU box).

Outputs (committed, data only):
  kat.json      -- the known-answer frames of TestPacket.java (hex literals), with the checksum
                   values that test pins (asserted or embedded in the frames it round-trips).
  pcap/*.pcap   -- the reference's pcap fixtures (test/src/test/resources/pcap/, MIT), copied
                   byte for byte as data.
  pcap_tuples.json -- the flow tuples TestPcap.java expects of each pcap frame (PktCheck lists:
                   src / dst address and port, and the TCP flags each PktCheck declares; the BSD
                   loopback test's ICMP address pairs), frame by frame.
  nat.json      -- the reference's own checkPartialAndModify rewrites of the KAT frames
                   (TestPacket.java:137-181, the setSrc / setDst / setTtl / setHopLimit /
                   setSrcPort / setDstPort calls of each KAT test) and IPInputRoute's TTL decrement,
                   with the expected bytes of the oracle's Java-semantics full recompute.

Usage:  python tests/golden/make_golden.py [/root/reference]
"""
from __future__ import annotations

import json
import os
import re
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

TESTPACKET = "test/src/test/java/io/vproxy/test/cases/TestPacket.java"
TESTPCAP = "test/src/test/java/io/vproxy/test/cases/TestPcap.java"
CONSTS = "base/src/main/java/io/vproxy/base/util/Consts.java"
PCAP_DIR = "test/src/test/resources/pcap"


def method_body(src: str, name: str) -> tuple[str, int, int]:
    m = re.search(r"public void " + re.escape(name) + r"\(\)\s*\{", src)
    assert m, name
    start = m.end()
    depth = 1
    i = start
    while depth:
        if src[i] == "{":
            depth += 1
        elif src[i] == "}":
            depth -= 1
        i += 1
    line0 = src[:m.start()].count("\n") + 1
    line1 = src[:i].count("\n") + 1
    return src[start:i], line0, line1


def bytes_from_calls(body: str, var: str) -> bytes:
    """Extract `var = ByteArray.from(0x.., ...)` or `ByteArray.fromHexString("..." + "...")`."""
    m = re.search(r"\b" + var + r"\s*=\s*ByteArray\.from\((.*?)\);", body, re.S)
    if m:
        vals = re.findall(r"0x([0-9a-fA-F]{1,2})", m.group(1))
        return bytes(int(v, 16) for v in vals)
    m = re.search(r"\b" + var + r"\s*=\s*ByteArray\.fromHexString\((.*?)\);", body, re.S)
    if m:
        return bytes.fromhex("".join(re.findall(r'"([0-9a-fA-F]*)"', m.group(1))))
    m = re.search(r"\bvar\s+" + var + r'\s*=\s*((?:"[0-9a-fA-F]*"\s*\+?\s*)+);', body, re.S)
    if m:
        return bytes.fromhex("".join(re.findall(r'"([0-9a-fA-F]*)"', m.group(1))))
    raise AssertionError(var)


def pcap_tuples(ref: str) -> dict:
    """TestPcap.java's expectations, frame by frame: the PktCheck lists of ether() and
    linuxCooked() (IPPort src, IPPort dst, TCP flags) and bsd()'s getSrc / getDst asserts."""
    src = open(os.path.join(ref, TESTPCAP)).read()
    consts = open(os.path.join(ref, CONSTS)).read()
    tcp_flag = {m.group(1): int(m.group(2), 2)
                for m in re.finditer(r"TCP_FLAGS_(\w+)\s*=\s*0b([01]+);", consts)}
    assert set(tcp_flag) >= {"SYN", "ACK", "PSH", "FIN", "RST"}
    ipport = r'new IPPort\("([^"]+)",\s*(\d+)\)'
    out = {}
    for meth, pcap in (("ether", "cap-ether.pcap"), ("linuxCooked", "cap-linux-cooked.pcap")):
        body, a, b = method_body(src, meth)
        assert f'"/pcap/{pcap}"' in body
        addrs = {m.group(1): (m.group(2), int(m.group(3)))
                 for m in re.finditer(r"var\s+(\w+)\s*=\s*" + ipport + ";", body)}
        rows = []
        line0 = a + body[:body.index("List.of(")].count("\n")
        for m in re.finditer(r"new PktCheck\((.*?)\)(?=,\s*\n|\s*\n\s*\))", body, re.S):
            args = m.group(1)
            ends = []
            for tok in re.finditer(ipport + "|" + r"\b(addr\d+)\b", args):
                ends.append((tok.group(1), int(tok.group(2))) if tok.group(1) else addrs[tok.group(3)])
            assert len(ends) == 2, args
            flags = 0
            for f in re.findall(r"Consts\.TCP_FLAGS_(\w+)", args):
                flags |= tcp_flag[f]
            ln = a + body[:m.start()].count("\n")
            rows.append(dict(src=ends[0][0], sport=ends[0][1], dst=ends[1][0], dport=ends[1][1], tcp_flags=flags,
                             source=f"{TESTPCAP}:{ln}"))
        out[pcap] = dict(method=f"{TESTPCAP}:{a}-{b}", asserted="src/dst address and port (check(), "
                         "TestPcap.java:16-30); tcp_flags are declared in each PktCheck but not asserted there",
                         frames=rows)
    body, a, b = method_body(src, "bsd")
    pairs = {}
    for m in re.finditer(r'assertEquals\(IP\.from\("([^"]+)"\),\s*pkts\.get\((\d+)\)\.get(Src|Dst)\(\)\)', body):
        pairs.setdefault(int(m.group(2)), {})[m.group(3).lower()] = m.group(1)
    assert "instanceof IcmpPacket" in body
    out["cap-bsd-loopback-encap.pcap"] = dict(
        method=f"{TESTPCAP}:{a}-{b}", asserted="src/dst address; every payload an IcmpPacket",
        frames=[dict(src=pairs[i]["src"], dst=pairs[i]["dst"], proto=1) for i in sorted(pairs)])
    assert [len(v["frames"]) for v in out.values()] == [13, 14, 4]
    return out


def main(ref: str) -> None:
    with open(os.path.join(HERE, "pcap_tuples.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (PktCheck lists parsed from TestPcap.java, TCP "
                                "flag values from Consts.java:56-61)", "pcaps": pcap_tuples(ref)}, f, indent=1)
    src = open(os.path.join(ref, TESTPACKET)).read()
    kats = []

    body, a, b = method_body(src, "ipv4ByIcmpExample")
    kats.append(dict(name="ipv4ByIcmpExample", source=f"{TESTPACKET}:{a}-{b}", layer="l3",
                     hex=bytes_from_calls(body, "bytes").hex(),
                     pinned={"ip": 0x76B8, "l4": 0x4D5A}, proto=1, ver=4))

    body, a, b = method_body(src, "ipv6ByIcmpExample")
    kats.append(dict(name="ipv6ByIcmpExample", source=f"{TESTPACKET}:{a}-{b}", layer="l3",
                     hex=bytes_from_calls(body, "bytes").hex(),
                     pinned={"l4": 0xD4EC}, proto=58, ver=6))

    body, a, b = method_body(src, "tcpIpv4SynExample")
    assert "assertEquals(0xf3ff, tcp.getChecksum())" in body
    kats.append(dict(name="tcpIpv4SynExample", source=f"{TESTPACKET}:{a}-{b}", layer="ether",
                     hex=bytes_from_calls(body, "bytes").hex(),
                     pinned={"ip": 0x87E4, "l4": 0xF3FF}, proto=6, ver=4))

    body, a, b = method_body(src, "tcpIpv4PshExample")
    assert "assertEquals(0x0aa9, tcp.getChecksum())" in body
    frame = bytes_from_calls(body, "header") + bytes_from_calls(body, "dataPart")
    kats.append(dict(name="tcpIpv4PshExample", source=f"{TESTPACKET}:{a}-{b}", layer="ether",
                     hex=frame.hex(), pinned={"ip": 0x85F7, "l4": 0x0AA9}, proto=6, ver=4))

    body, a, b = method_body(src, "udpIpv4Example")
    assert "assertEquals(0xdf0d, udp.getChecksum())" in body
    frame = bytes_from_calls(body, "header") + bytes_from_calls(body, "data")
    kats.append(dict(name="udpIpv4Example", source=f"{TESTPACKET}:{a}-{b}", layer="ether",
                     hex=frame.hex(), pinned={"ip": 0x7F41, "l4": 0xDF0D}, proto=17, ver=4))

    body, a, b = method_body(src, "etherip")
    frame = bytes_from_calls(body, "hex")
    # outer IPv4 (proto 97 EtherIP) at 14; inner Ethernet at 14+20+2; inner IPv4 at +14; ICMP.
    kats.append(dict(name="etherip", source=f"{TESTPACKET}:{a}-{b}", layer="ether",
                     hex=frame.hex(), pinned={"ip": 0xFC82, "inner_ip": 0x2C7A, "inner_l4": 0xEE43},
                     proto=97, ver=4, inner_l3_off=14 + 20 + 2 + 14))

    # sanity: pinned values are literally present in the frames
    for k in kats:
        fr = bytes.fromhex(k["hex"])
        for v in k["pinned"].values():
            assert v.to_bytes(2, "big") in fr, (k["name"], hex(v))

    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "kats": kats}, f, indent=1)

    os.makedirs(os.path.join(HERE, "pcap"), exist_ok=True)
    for fn in sorted(os.listdir(os.path.join(ref, PCAP_DIR))):
        if fn.endswith(".pcap"):
            shutil.copyfile(os.path.join(ref, PCAP_DIR, fn), os.path.join(HERE, "pcap", fn))

    # NAT rewrites: the reference's own checkPartialAndModify calls (TestPacket.java:137-181 and
    # the lines below), parsed from the test source, plus the TTL decrement of IPInputRoute
    # (core/.../vswitch/node/IPInputRoute.java:79-91).  Expected bytes: the oracle's
    # Java-semantics rewrite + full recompute (oracle/csum_oracle.c:orc_nat_java).
    import ipaddress
    from oracle import oracle as O
    import numpy as np
    lines = src.split("\n")
    calls = []
    for ln, text in enumerate(lines, 1):
        if "checkPartialAndModify(" in text and "void checkPartialAndModify" not in text:
            call = text + (lines[ln] if text.rstrip().endswith(",") else "")
            calls.append((ln, call))
    methods = {k["name"]: method_body(src, k["name"])[1:] for k in kats}

    def rewrite_of(call: str):
        m = re.search(r"set(Src|Dst)\(\(IPv[46]\) IP\.from\(\"([^\"]+)\"\)\)", call)
        if m:
            return ("NAT_" + m.group(1).upper(), ipaddress.ip_address(m.group(2)).packed)
        m = re.search(r"\.(setTtl|setHopLimit)\((\d+)\)", call)
        if m:
            return ("NAT_SET_TTL", int(m.group(2)))
        m = re.search(r"\.set(Src|Dst)Port\((\d+)\)", call)
        if m:
            return ("NAT_" + m.group(1).upper()[0] + "PORT", int(m.group(2)))
        return None

    def entry(kind, val):
        rw = np.zeros(1, O.NAT_DTYPE)
        if kind in ("NAT_SRC", "NAT_DST"):
            rw[0][kind[4:].lower()][:len(val)] = list(val)
        elif kind == "NAT_SET_TTL":
            rw[0]["ttl"] = val
        elif kind in ("NAT_SPORT", "NAT_DPORT"):
            rw[0][kind[4:].lower()] = [val >> 8, val & 0xFF]
        rw[0]["mask"] = getattr(O, kind)
        return rw

    nat_cases = []
    orc = O.Oracle()
    for k in kats:
        a, b = methods[k["name"]]
        mine = [(ln, c) for ln, c in calls if a <= ln <= b]
        label = {"NAT_SRC": "setSrc({})", "NAT_DST": "setDst({})", "NAT_SET_TTL": "setTtl / setHopLimit({})",
                 "NAT_SPORT": "setSrcPort({})", "NAT_DPORT": "setDstPort({})"}
        todo = []
        for ln, c in mine:
            r = rewrite_of(c)
            if r is not None:
                v = str(ipaddress.ip_address(r[1])) if r[0] in ("NAT_SRC", "NAT_DST") else r[1]
                todo.append((f"{TESTPACKET}:{ln}", label[r[0]].format(v), r))
        if k["ver"] == 4 and k["proto"] in (1, 6, 17):
            todo.append(("core/src/main/java/io/vproxy/vswitch/node/IPInputRoute.java:79-91",
                         "TTL decrement (setTtl(ttl - 1))", ("NAT_DEC_TTL", None)))
        fr = bytes.fromhex(k["hex"])
        l3off = 0 if k["layer"] == "l3" else 14
        info, err = O.parse_l3(fr, l3off, len(fr) - l3off)
        assert err is None
        for srcline, text, (kind, val) in todo:
            arena = np.frombuffer(fr, np.uint8).copy()
            desc = np.zeros(1, O.DESC_DTYPE)
            desc[0] = (info.l3_off, info.l3_len, info.l4_off, info.ver, info.proto, O.desc_flags_for(info), 0)
            rw = entry(kind, val)
            st = orc.nat_java(arena, desc, rw)
            assert st[0] == O.S_DONE
            nat_cases.append(dict(kat=k["name"], ver=info.ver, rewrite=text, source=srcline, mask=int(rw[0]["mask"]),
                                  entry=rw.tobytes().hex(), l3_off=l3off, before=fr.hex(),
                                  after=arena.tobytes().hex()))
    assert sum(c["source"].startswith(TESTPACKET) for c in nat_cases) == 18   # 3 + 3 + 4 x 3
    with open(os.path.join(HERE, "nat.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (rewrites parsed from TestPacket.java; expected "
                                "bytes from the oracle's Java-semantics full recompute)",
                   "entry": "vpcsum_nat_t (48 B, include/vpcsum.h), hex",
                   "cases": nat_cases}, f, indent=1)
    print(f"kats={len(kats)} nat={len(nat_cases)}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
