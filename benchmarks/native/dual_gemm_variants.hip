// Standalone timing of one compile-time variant of the dual GEMM (DG_PD set on the
// hipcc line). Random bf16 operands; prints ms and effective TB/s per shape.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../csrc/kernels/dual_gemm.hip"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void fill(uint16_t* p, int64_t n, uint32_t seed) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
    float f = ((x & 0xffff) / 65536.0f - 0.5f);
    p[i] = dgraph::f32_to_bf16(f);
  }
}

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atoll(argv[1]) : (1 << 25);
  const int shapes[][3] = {{256, 128, 128}, {256, 256, 256}, {256, 192, 192}, {192, 256, 0}};
  uint16_t *A1, *A2, *B1, *B2, *out;
  uint64_t* mask;
  CK(hipMalloc(&A1, M * 256 * 2)); CK(hipMalloc(&A2, M * 256 * 2));
  CK(hipMalloc(&B1, 256 * 256 * 2)); CK(hipMalloc(&B2, 256 * 256 * 2));
  CK(hipMalloc(&out, M * 256 * 2)); CK(hipMalloc(&mask, (M + 255) / 256 * 8 * 8 * 16 * 8));
  fill<<<4096, 256>>>(A1, M * 256, 1); fill<<<4096, 256>>>(A2, M * 256, 2);
  fill<<<256, 256>>>(B1, 256 * 256, 3); fill<<<256, 256>>>(B2, 256 * 256, 4);
  CK(hipDeviceSynchronize());
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  for (auto& sh : shapes) {
    const int N = sh[0], K1 = sh[1], K2 = sh[2];
    auto run = [&]() {
      CK(dgraph::dual_gemm(A1, K1, B1, K1, K2 ? A2 : nullptr, K2, B2, K2, nullptr, nullptr, 0,
                           out, N, M, N, K2 ? mask : nullptr, nullptr, K2 > 0, 0));
    };
    run(); CK(hipDeviceSynchronize());
    hipEventRecord(s);
    for (int i = 0; i < 5; ++i) run();
    hipEventRecord(e); hipEventSynchronize(e);
    float ms; hipEventElapsedTime(&ms, s, e); ms /= 5;
    double bytes = (double)M * (K1 + K2 + N) * 2;
    printf("PD=%d N=%d K1=%d K2=%d: %.2f ms %.2f TB/s\n", DG_PD, N, K1, K2, ms,
           bytes / ms / 1e9);
  }
  return 0;
}
