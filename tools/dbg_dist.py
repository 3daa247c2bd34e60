import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests", "golden"))
import numpy as np
import inputs
from kman_amd import dist, engine
nb = int(sys.argv[1])
text = inputs.syn_numpy(nb, 1)
dev = engine.Device(0)
p = dist.DistPipeline(dev, text, 21, "uniq", 1, 0, dist.unique_id())
print("path after init", p.path, "nbq", p.n_bases_q, flush=True)
g = p._region_step()
req = next(g)
while True:
    print("req", req[0], flush=True)
    try:
        if req[0] == "allreduce": req = g.send(p.comm.allreduce(req[1]))
        elif req[0] == "allgather":
            out = p.comm.allgather(req[1]); print("counts sum", out.sum(), out[0][:4]); req = g.send(out)
        else:
            p.comm.alltoallv(*req[1]); dev.sync()
            for off in (100_000_000, 140_000_000, 160_000_000, 200_000_000, 290_000_000):
                s2 = dev.download(p.send, 1000, np.uint64, offset=8 * off); r2 = dev.download(p.recv, 1000, np.uint64, offset=8 * off)
                print("off", off, "send nonzero", int((s2 != 0).sum()), "recv nonzero", int((r2 != 0).sum()), "eq", bool((s2 == r2).all()), flush=True)
            s = dev.download(p.send, 4_000_000, np.uint64); r = dev.download(p.recv, 4_000_000, np.uint64)
            print("send==recv", bool((s == r).all()), "bit63 frac", float(((s >> np.uint64(63)) & np.uint64(1)).mean()),
                  "top9 of first bucket", np.bincount((s[:100000] >> np.uint64(55)).astype(np.int64), minlength=512)[:8],
                  "max pos", int((s & np.uint64((1 << 30) - 1)).max()), flush=True)
            req = g.send(None)
    except StopIteration as e:
        print("result", e.value, flush=True); break
