import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from oracle import oracle as O
from vproxy_amd import vpcsum as V
orc = O.Oracle()
for wl in (1,2,3):
  for team in (0,2,6):
    n=3000; stride=1536
    a, d = orc.synth(n, stride, 0, wl, O.SEED, 12345)
    arena = torch.from_numpy(a.copy()).cuda(); dt = V.desc_to_tensor(d)
    out = torch.zeros(n, dtype=torch.int32, device='cuda'); st = torch.zeros(n, dtype=torch.uint8, device='cuda')
    V.compute(arena, dt, n, out, st, V.MODE_WRITE, team); torch.cuda.synchronize()
    w = arena.cpu().numpy(); a2 = a.copy(); orc.process(a2, d, 0, write=True)
    diff = np.nonzero(w != a2)[0]
    print(wl, team, len(diff), diff[:10], [(int(x)//stride, int(x)%stride, a[x], w[x], a2[x]) for x in diff[:6]])
