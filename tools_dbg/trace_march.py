# Oracle march trace of one pixel of the synthetic C3/C4 scenes (debug helper).
import sys, numpy as np, ctypes
sys.path[:0] = ['3dg-vol-renderer_amd', 'oracle', 'tests', '.']
import pyoracle as O
from test_gpu_parity import _synthetic_scene
from helpers import CAM_POS, FOV, main_view_dir
W, H, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
x, y = int(sys.argv[4]), int(sys.argv[5])
scene, osc = _synthetic_scene(n)
L = O.lib(); f = L.orc_debug_march; f.restype = ctypes.c_int64
FP = ctypes.POINTER(ctypes.c_float)
f.argtypes = [ctypes.c_void_p, FP, FP, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
              ctypes.c_float, ctypes.c_int, FP, FP, ctypes.c_int64]
out = np.zeros(1000000, np.float32)
pos = np.ascontiguousarray(CAM_POS, np.float32); vd = np.ascontiguousarray(main_view_dir(), np.float32)
Lo = np.zeros(3, np.float32)
m = f(osc.h, pos.ctypes.data_as(FP), vd.ctypes.data_as(FP), FOV, x, y, W, H, 0.01, int(sys.argv[6]), Lo.ctypes.data_as(FP), out.ctypes.data_as(FP), out.size)
print('L', Lo, 'render', O.render(osc, O.PINHOLE, CAM_POS, main_view_dir(), FOV, W, H, O.RAYMARCH_GAUSSIANS, 0.01, int(sys.argv[6]), pixels=np.array([[x, y]], np.int32)))
i = 0
while i < m:
    t, na, ss, T = out[i:i + 4]; ids = out[i + 4:i + 4 + int(na)].astype(int); i += 4 + int(na)
    print('t=%.7f n=%d ss=%.4g T=%.6g' % (t, na, ss, T), ids)
