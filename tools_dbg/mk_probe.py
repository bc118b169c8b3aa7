import sys, numpy as np
sys.path[:0] = ['3dg-vol-renderer_amd', 'oracle', 'tests']
import pyoracle as O
from helpers import scene_path
rng = np.random.default_rng(0)
s = O.OracleScene.load_gmm(scene_path('50_random.txt'))
rec = s.records()  # mean3 dens inv6 norm alb
n = 200000
gi = rng.integers(0, rec.shape[0], n)
R = rec[gi]
# device record layout: mx my mz dens m00 m01 m02 m11 m12 m22 norm alb  (same order)
o = (R[:, :3] + rng.normal(scale=0.6, size=(n, 3))).astype(np.float32)
d = rng.normal(size=(n, 3)); d /= np.linalg.norm(d, axis=1, keepdims=True); d = d.astype(np.float32)
xi = (rng.integers(0, 1 << 24, (n, 2)) * (1.0 / 16777216.0)).astype(np.float32)
with open('tools_dbg/probe_in.bin', 'wb') as f:
    f.write(np.int32(n).tobytes()); f.write(R.astype(np.float32).tobytes()); f.write(np.hstack([o, d]).astype(np.float32).tobytes()); f.write(xi.tobytes())
np.save('tools_dbg/probe_meta.npy', gi)
