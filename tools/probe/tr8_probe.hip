#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(2))) int i32x2;
typedef __attribute__((ext_vector_type(4))) short s16x4;
// LDS image: byte at offset a = a & 0xff pattern via 16-bit (row, col): we fill LDS bytes with index (a) and read back
__global__ void probe(int* out, int mode, int stride) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[8192];
  for (int i = threadIdx.x; i < 8192; i += 64) lds[i] = 0;
  __syncthreads();
  // fill: 64 rows of `stride` bytes; byte (r, c) = r*? -> store row in high nibble? use 16-bit ids via two passes
  for (int i = threadIdx.x; i < 8192; i += 64) lds[i] = (mode == 0) ? (i / stride) : (i % stride);
  __syncthreads();
  const int lane = threadIdx.x;
  typedef __attribute__((address_space(3))) i32x2 lds_i32x2;
  // each lane points at row (lane) ? use address = lane * stride (row = lane) 
  const unsigned char* p = lds + (lane * stride) % 8192;
  i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i32x2*)(p));
  out[lane * 2] = v[0];
  out[lane * 2 + 1] = v[1];
}
int main() {
  int* d; hipMalloc(&d, 64 * 2 * 4);
  int h[128];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode, 64);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("mode %d (%s):\n", mode, mode == 0 ? "row id" : "byte-in-row");
    for (int l = 0; l < 64; ++l) {
      unsigned char* b = (unsigned char*)&h[l * 2];
      printf("L%02d:", l);
      for (int j = 0; j < 8; ++j) printf(" %3d", b[j]);
      printf(l % 2 ? "\n" : "   ");
    }
  }
  return 0;
}
