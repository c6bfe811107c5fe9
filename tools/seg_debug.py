"""Debug: config-5 frames (first N) through a geometry vs the oracle; prints
the mismatching frame indices (unit = index / 64, lane = index % 64)."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import bench, oracle
import libxudp_amd as X

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
geoms = [tuple(map(int, g.split(","))) for g in (sys.argv[2] if len(sys.argv) > 2 else "64,64,4;64,1,9").split(";")]
cfg = bench.CONFIGS[5]
umem, desc = X.gen_frames_host(n, 4, cfg["pmin"], cfg["pmax"], seed=bench.SEED_BASE ^ 5)
exp = oracle.batch(umem, desc, cfg["mode"])
eng = X.Engine(0)
dev = torch.device("cuda:0")
d_umem = torch.from_numpy(umem).to(dev)
d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
bpcs = [int(b) for b in (sys.argv[3] if len(sys.argv) > 3 else '0').split(',')]
for g, bpc in [(g, b) for g in geoms for b in bpcs]:
    eng.set_geometry(*g)
    eng.set_launch(bpc)
    out = torch.zeros(n, dtype=torch.int16, device=dev)
    eng.batch_device(d_umem, d_desc, n, out, cfg["mode"], 0, 4500)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint16)
    bad = np.nonzero(got != exp)[0]
    print(g, "bpc", bpc, "n", n, "bad", len(bad), "first", bad[:20].tolist(), "units", sorted(set((bad // 64).tolist()))[:20], flush=True)
    if len(bad):
        i = bad[0]
        print("  lanes of first bad unit:", sorted((bad[bad // 64 == i // 64] % 64).tolist()))
eng.set_geometry(0)
