// Probe of v_cvt_pk_u8_f32's conversion on gfx950: rounding of halves and saturation, so an int8
// quantiser can hand it a non-integer float.  Build: hipcc --offload-arch=gfx950 -O2 -o
// tools/probe_cvt_u8 tools/probe_cvt_u8.hip; run on the GPU box.  Prints x -> byte for each probe.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__global__ void probe(const float* x, unsigned* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = __builtin_amdgcn_cvt_pk_u8_f32(x[i], 0, 0u);
}

int main() {
  const float xs[] = {0.0f, 0.49f, 0.5f, 0.51f, 1.5f, 2.5f, 3.5f, 126.5f, 127.5f, 128.5f, 254.5f, 255.0f,
                      255.4f, 255.5f, 256.0f, 300.0f, 1e9f, -0.4f, -0.5f, -0.6f, -1.0f, -300.0f, -1e9f,
                      NAN, INFINITY, -INFINITY, 129.49999f, 129.50001f};
  const int n = sizeof(xs) / sizeof(xs[0]);
  float* dx;
  unsigned* dout;
  unsigned out[64];
  if (hipMalloc(&dx, sizeof(xs)) || hipMalloc(&dout, n * 4)) return 1;
  if (hipMemcpy(dx, xs, sizeof(xs), hipMemcpyHostToDevice)) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dx, dout, n);
  if (hipDeviceSynchronize() || hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost)) return 1;
  for (int i = 0; i < n; ++i) printf("cvt_pk_u8(%.7g) = %u\n", xs[i], out[i] & 0xFFu);
  return 0;
}
