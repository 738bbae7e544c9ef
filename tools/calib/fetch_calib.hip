// Calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access shapes the swarm step uses
// (4-byte-per-lane coalesced SoA loads/stores, 16-byte-per-lane obs tile stores), on a known byte
// count: each kernel touches exactly BYTES bytes once.  Run under rocprofv3 --pmc FETCH_SIZE (and a
// separate WRITE_SIZE pass); tools/summarize_prof.py turns the ratios into correction factors.
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr size_t BYTES = 256ull << 20;   // 256 MiB: well past the 32 MiB of L2

__global__ void read_b32(const float* __restrict__ a, float* out, size_t n) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.f) out[0] = s;
}
__global__ void read_b128(const float4* __restrict__ a, float* out, size_t n4) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;
}
__global__ void write_b32(float* a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = 1.f;
}
__global__ void write_b128(float4* a, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

// The step kernel's state-word shape (flavor B, 4 sub-lanes per drone, 16 drones per wave): sub-lane q of drone g
// touches words q, q + 4, ... of the SoA field block [W][I], i.e. every load / store instruction covers four 64-B
// row segments; blocks of one wave, mapped to XCDs like the step (<true>, xcd_block: a contiguous run of drones per
// XCD, so the two 64-B halves of a 128-B line meet in one L2) or round-robin (<false>: the halves land in two L2s).
constexpr int SUB_W = 64;                          // words per drone
constexpr size_t SUB_I = BYTES / (4 * SUB_W);      // drones
__device__ __forceinline__ int xcd_block(int b, int nb) { return (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3); }
template <bool XCD>
__global__ void read_sub64(const float* __restrict__ a, float* out) {
    const int blk = XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const size_t g = (size_t)blk * 16 + threadIdx.x / 4;
    const int q = threadIdx.x % 4;
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < SUB_W / 4; ++t) s += a[(size_t)(q + 4 * t) * SUB_I + g];
    if (s == 12345.f) out[0] = s;
}
template <bool XCD>
__global__ void write_sub64(float* a) {
    const int blk = XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const size_t g = (size_t)blk * 16 + threadIdx.x / 4;
    const int q = threadIdx.x % 4;
#pragma unroll
    for (int t = 0; t < SUB_W / 4; ++t) a[(size_t)(q + 4 * t) * SUB_I + g] = (float)t;
}

int main() {
    float *a, *o;
    if (hipMalloc(&a, BYTES) != hipSuccess || hipMalloc(&o, 256) != hipSuccess) return 1;
    (void)hipMemset(a, 0, BYTES);
    const size_t n = BYTES / 4;
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(read_b32, dim3(4096), dim3(256), 0, 0, a, o, n);
        hipLaunchKernelGGL(read_b128, dim3(4096), dim3(256), 0, 0, (const float4*)a, o, n / 4);
        hipLaunchKernelGGL(write_b32, dim3(4096), dim3(256), 0, 0, a, n);
        hipLaunchKernelGGL(write_b128, dim3(4096), dim3(256), 0, 0, (float4*)a, n / 4);
        hipLaunchKernelGGL(read_sub64<true>, dim3(SUB_I / 16), dim3(64), 0, 0, a, o);
        hipLaunchKernelGGL(read_sub64<false>, dim3(SUB_I / 16), dim3(64), 0, 0, a, o);
        hipLaunchKernelGGL(write_sub64<true>, dim3(SUB_I / 16), dim3(64), 0, 0, a);
        hipLaunchKernelGGL(write_sub64<false>, dim3(SUB_I / 16), dim3(64), 0, 0, a);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("calib bytes per kernel %zu\n", BYTES);
    (void)hipFree(a);
    (void)hipFree(o);
    return 0;
}
