import sys, json, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from oracle import oracle as O
from vproxy_amd import vpcsum as V
d = json.load(open('tests/golden/nat.json'))
c = [c for c in d['cases'] if c['kat']=='udpIpv4Example' and c['rewrite']=='setSrc'][0]
fr = bytearray(bytes.fromhex(c['before']))
fr[14+12:14+16] = bytes([1,2,3,4])   # CPU-side rewrite
info,_ = O.parse_l3(bytes(fr), 14, len(fr)-14)
desc = np.array([(14, info.l3_len, info.l4_off, 4, info.proto, 3, 0)], dtype=O.DESC_DTYPE)
orc = O.Oracle()
a = np.frombuffer(bytes(fr), np.uint8).copy()
want, _ = orc.process(a.copy(), desc)
print('oracle', hex(want[0]))
for v in (3, 9, 21, 26, 0):
    for mode in (0, 1, 0x10):
        t = torch.from_numpy(a.copy()).cuda(); dt = V.desc_to_tensor(desc)
        o = torch.zeros(1, dtype=torch.int32, device='cuda'); s = torch.zeros(1, dtype=torch.uint8, device='cuda')
        V.compute(t, dt, 1, o, s, mode, v); torch.cuda.synchronize()
        print(v, mode, hex(int(o.cpu().numpy().view(np.uint32)[0])), s.cpu().numpy())
# also padded arena (len multiple of 16)
for padlen in (len(fr), 128, 4096):
    b = np.zeros(padlen, np.uint8); b[:len(fr)] = a
    t = torch.from_numpy(b).cuda(); dt = V.desc_to_tensor(desc)
    o = torch.zeros(1, dtype=torch.int32, device='cuda')
    V.compute(t, dt, 1, o, None, 0, 26); torch.cuda.synchronize()
    print('arena', padlen, hex(int(o.cpu().numpy().view(np.uint32)[0])))
