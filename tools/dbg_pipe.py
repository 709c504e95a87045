import sys, numpy as np
sys.path.insert(0, "/root/repo")
import mpi_cuda_imagemanipulation_amd as m
C = m._C
for chain in ["blur:9", "blur:3", "gaussian5"]:
  for ranks, H, it in [(2, 96, 4), (2, 96, 1), (2, 96, 2), (4, 130, 4)]:
    img = m.utils.synthetic_image(7, 203, H, 3)
    res = []
    for pipeline, nr in ((True, ranks), (False, ranks), (True, 1)):
        cfg = m.Pipeline(chain).config(203, H, 3, "device", device=0)
        cfg.pipeline = pipeline
        res.append(C.run_local_group(cfg, nr, img, it).astype(int))
    d01 = np.argwhere(res[0] != res[2]); d12 = np.argwhere(res[1] != res[2])
    print(chain, ranks, H, it, "pipe-vs-1rank", len(d01), "rows", sorted(set(d01[:, 0].tolist()))[:20],
          "plain-vs-1rank", len(d12), "rows", sorted(set(d12[:, 0].tolist()))[:20], flush=True)
