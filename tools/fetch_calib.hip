// FETCH_SIZE calibration for gather access patterns (VERDICT r04 "next" item 2).
//
// The guide (MI355X_MICROARCH.md, HBM section) calibrates rocprofv3 FETCH_SIZE only for 16-B/lane
// coalesced streaming reads (it reports half the bytes). The classification kernels make scattered
// 4-16-B gathers, so this program reads KNOWN sets of distinct 128-B lines in random order with
// 4-, 8- and 16-B loads per lane and prints the bytes each launch must move; run it under
//   rocprofv3 --pmc FETCH_SIZE ...            (one pass)
//   rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum ...
// and divide (tools/fetch_calib.py does both passes and writes the table).
//
// Kernels (one launch each, distinct names so the counter CSV separates them):
//   stream16    coalesced 16 B / lane over the whole buffer (the guide's calibrated case)
//   gatherW_L   one lane = one W-byte load from a distinct 128-B line (line index = a bijection of
//               the lane id over 2^k lines, so every line of the buffer's first 2^k lines is read
//               exactly once, in scattered order); W in {4, 8, 16}
//   gather16x8  8 lanes read one whole 128-B line (16 B each), lines in scattered order
//   gather4_rep each lane reads 4 B from a line, every line read by 4 lanes of different waves
// The buffer is 128 MiB (Infinity-Cache resident, like the C3 image) or 1 GiB (HBM) by argv.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

constexpr uint32_t kLine = 128;

__device__ __forceinline__ uint64_t scatter_line(uint64_t i, uint32_t lg) {  // bijection on [0, 2^lg)
  const uint64_t m = (1ull << lg) - 1;  // odd multiplies and xor-shifts mod 2^lg are bijections
  uint64_t x = (i * 0x9E3779B97F4A7C15ull) & m;
  x ^= x >> (lg / 2);
  return (x * 0xBF58476D1CE4E5B9ull) & m;
}

__global__ void stream16(const uint4* __restrict__ buf, uint64_t n16, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint4 v = buf[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int W>
__device__ __forceinline__ void gather_line(const uint8_t* __restrict__ buf, uint32_t lg, uint32_t* __restrict__ sink) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= (1ull << lg)) return;
  const uint8_t* p = buf + scatter_line(i, lg) * kLine;
  uint32_t acc;
  if constexpr (W == 4) {
    acc = *reinterpret_cast<const uint32_t*>(p);
  } else if constexpr (W == 8) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    acc = v.x ^ v.y;
  } else {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    acc = v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void gather4_L(const uint8_t* b, uint32_t lg, uint32_t* s) { gather_line<4>(b, lg, s); }
__global__ void gather8_L(const uint8_t* b, uint32_t lg, uint32_t* s) { gather_line<8>(b, lg, s); }
__global__ void gather16_L(const uint8_t* b, uint32_t lg, uint32_t* s) { gather_line<16>(b, lg, s); }

__global__ void gather16x8(const uint4* __restrict__ buf, uint32_t lg, uint32_t* __restrict__ sink) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= (8ull << lg)) return;
  const uint4 v = buf[scatter_line(i >> 3, lg) * 8 + (i & 7)];
  const uint32_t acc = v.x ^ v.y ^ v.z ^ v.w;
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void gather4_rep(const uint8_t* __restrict__ buf, uint32_t lg, uint32_t* __restrict__ sink) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= (4ull << lg)) return;
  // copy r of line j is read by lane (r << lg) + j: the copies sit in different waves
  const uint64_t j = i & ((1ull << lg) - 1);
  const uint32_t r = uint32_t(i >> lg);
  const uint32_t acc = *reinterpret_cast<const uint32_t*>(buf + scatter_line(j, lg) * kLine + 4 * r);
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 128;
  const uint64_t bytes = mib << 20;
  uint32_t lg = 0;
  while ((uint64_t(kLine) << (lg + 1)) <= bytes) lg++;
  uint8_t* buf;
  uint32_t* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 256));
  CK(hipMemset(buf, 0x5a, bytes));
  CK(hipDeviceSynchronize());
  const uint64_t lines = 1ull << lg;
  auto blocks = [](uint64_t n) { return dim3(uint32_t((n + 255) / 256)); };
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](const char* name, uint64_t known, auto fn) {
    fn();  // warm (Infinity Cache fill)
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    fn();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("%s\t%llu\t%.4f\n", name, (unsigned long long)known, ms);
  };
  std::printf("# buffer %llu MiB, %llu lines of 128 B; columns: kernel, distinct bytes per launch, ms\n",
              (unsigned long long)mib, (unsigned long long)lines);
  timed("stream16", bytes, [&] { hipLaunchKernelGGL(stream16, dim3(2048), dim3(256), 0, 0, (const uint4*)buf, bytes / 16, sink); });
  timed("gather4_L", lines * kLine, [&] { hipLaunchKernelGGL(gather4_L, blocks(lines), dim3(256), 0, 0, buf, lg, sink); });
  timed("gather8_L", lines * kLine, [&] { hipLaunchKernelGGL(gather8_L, blocks(lines), dim3(256), 0, 0, buf, lg, sink); });
  timed("gather16_L", lines * kLine, [&] { hipLaunchKernelGGL(gather16_L, blocks(lines), dim3(256), 0, 0, buf, lg, sink); });
  timed("gather16x8", lines * kLine, [&] { hipLaunchKernelGGL(gather16x8, blocks(8 * lines), dim3(256), 0, 0, (const uint4*)buf, lg, sink); });
  timed("gather4_rep", lines * kLine, [&] { hipLaunchKernelGGL(gather4_rep, blocks(4 * lines), dim3(256), 0, 0, buf, lg, sink); });
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
