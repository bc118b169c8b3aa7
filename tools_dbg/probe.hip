// Debug: evaluate device intersect / optical depth / env_dir / primary ray for host-supplied inputs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <fstream>
#include "../3dg-vol-renderer_amd/csrc/kernels/vr_march.h"
using namespace vr; using namespace vr::dev;
__global__ void k_probe(const GaussianRecord* g, const float* rays, int n, float* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
  const float* r = rays + 6 * i;
  Ray ray{r[0], r[1], r[2], r[3], r[4], r[5]};
  GRec gr = load_rec(g, i);
  Quad q = quad(gr, ray);
  float a = 0, b = 0; bool hit = intersect(q, a, b);
  out[8*i+0] = hit; out[8*i+1] = a; out[8*i+2] = b; out[8*i+3] = hit ? optical_depth(gr, q, a, b) : 0.f;
  out[8*i+4] = q.A; out[8*i+5] = q.B; out[8*i+6] = q.Cq; out[8*i+7] = mu_t(gr, r[0] + 0.1f, r[1], r[2]);
}
__global__ void k_env(const float* xi, int n, float* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
  float x, y, z; env_dir(xi[2*i], xi[2*i+1], x, y, z); normalize3(x, y, z);
  out[3*i] = x; out[3*i+1] = y; out[3*i+2] = z;
}
int main(int argc, char** argv) {
  std::ifstream f(argv[1], std::ios::binary); int n; f.read((char*)&n, 4);
  std::vector<GaussianRecord> g(n); std::vector<float> rays(6*n), xi(2*n);
  f.read((char*)g.data(), 48*n); f.read((char*)rays.data(), 24*n); f.read((char*)xi.data(), 8*n);
  GaussianRecord* dg; float *dr, *dout, *dxi, *denv;
  hipMalloc(&dg, 48*n); hipMalloc(&dr, 24*n); hipMalloc(&dout, 32*n); hipMalloc(&dxi, 8*n); hipMalloc(&denv, 12*n);
  hipMemcpy(dg, g.data(), 48*n, hipMemcpyHostToDevice); hipMemcpy(dr, rays.data(), 24*n, hipMemcpyHostToDevice);
  hipMemcpy(dxi, xi.data(), 8*n, hipMemcpyHostToDevice);
  k_probe<<<(n+255)/256, 256>>>(dg, dr, n, dout); k_env<<<(n+255)/256, 256>>>(dxi, n, denv);
  std::vector<float> out(8*n), env(3*n);
  hipMemcpy(out.data(), dout, 32*n, hipMemcpyDeviceToHost); hipMemcpy(env.data(), denv, 12*n, hipMemcpyDeviceToHost);
  std::ofstream o(argv[2], std::ios::binary); o.write((char*)out.data(), 32*n); o.write((char*)env.data(), 12*n);
  printf("probe done n=%d\n", n); return 0;
}
