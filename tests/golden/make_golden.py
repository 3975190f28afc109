"""Generate tests/golden/ fixtures from the reference's own test data (run in the build
container only; /root/reference does not exist on the GPU box).

Outputs (committed, data only):
  kat.json      -- the known-answer frames of TestPacket.java (hex literals), with the checksum
                   values that test pins (asserted or embedded in the frames it round-trips).
  pcap/*.pcap   -- the reference's pcap fixtures (test/src/test/resources/pcap/, MIT), copied
                   byte for byte as data.
  nat.json      -- checkPartialAndModify-style rewrites of the KAT frames (TestPacket.java:137-181)
                   with the expected bytes produced by the oracle's Java-semantics full recompute.

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


def main(ref: str) -> None:
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

    # NAT rewrites mirroring checkPartialAndModify (TestPacket.java:137-181): expected bytes from
    # the oracle's Java-semantics rewrite + full recompute.
    from oracle import oracle as O
    import numpy as np
    nat_cases = []
    rewrites = [("setSrc", O.NAT_SRC), ("setDst", O.NAT_DST), ("setSrcPort", O.NAT_SPORT),
                ("setDstPort", O.NAT_DPORT), ("setTtl", O.NAT_DEC_TTL)]
    orc = O.Oracle()
    for k in kats:
        if k["ver"] != 4 or k["proto"] not in (6, 17, 1):
            continue
        fr = bytes.fromhex(k["hex"])
        l3off = 0 if k["layer"] == "l3" else 14
        info, err = O.parse_l3(fr, l3off, len(fr) - l3off)
        assert err is None
        for rname, mask in rewrites:
            if k["proto"] == 1 and mask in (O.NAT_SPORT, O.NAT_DPORT):
                continue
            arena = np.frombuffer(fr, np.uint8).copy()
            desc = np.zeros(1, O.DESC_DTYPE)
            desc[0] = (info.l3_off, info.l3_len, info.l4_off, 4, info.proto, O.desc_flags_for(info), 0)
            rw = np.zeros(1, O.NAT4_DTYPE)
            rw[0]["src"] = [1, 2, 3, 4]
            rw[0]["dst"] = [1, 2, 3, 4]
            rw[0]["sport"] = [0, 121]
            rw[0]["dport"] = [0, 121]
            rw[0]["mask"] = mask
            orc.nat4_java(arena, desc, rw)
            nat_cases.append(dict(kat=k["name"], rewrite=rname, mask=mask, l3_off=l3off,
                                  before=fr.hex(), after=arena.tobytes().hex()))
    with open(os.path.join(HERE, "nat.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (oracle full recompute)",
                   "rewrite": {"src": "1.2.3.4", "dst": "1.2.3.4", "sport": 121, "dport": 121,
                               "ttl": "decrement (setTtl(ttl-1), IPInputRoute.java:79-91)"},
                   "cases": nat_cases}, f, indent=1)
    print(f"kats={len(kats)} nat={len(nat_cases)}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
