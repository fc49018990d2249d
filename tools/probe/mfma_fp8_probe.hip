// Probe of v_mfma_scale_f32_16x16x128_f8f6f4 operand/scale semantics: one wave, A/B fragments
// given per lane (32 bytes), D returned per lane (4 floats).
#include <hip/hip_runtime.h>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void k(const i32x8* a, const i32x8* b, f32x4* d, int sa, int sb, int which) {
  int l = threadIdx.x;
  f32x4 c = {0, 0, 0, 0};
  if (which == 0)
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], c, 0, 0, 0, 127, 0, 127);
  else if (which == 1)
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], c, 0, 0, 0, sa, 0, sb);
  else {
    typedef __attribute__((ext_vector_type(2))) int i32x2;
    i32x2 aa = {a[l][0], a[l][1]}, bb = {b[l][0], b[l][1]};
    c = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(__builtin_bit_cast(long, aa), __builtin_bit_cast(long, bb), c, 0, 0, 0);
  }
  d[l] = c;
}
extern "C" int probe(const void* a, const void* b, void* d, int sa, int sb, int which) {
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, (const i32x8*)a, (const i32x8*)b, (f32x4*)d, sa, sb, which);
  return hipDeviceSynchronize();
}
