// fetch_calib.hip -- what rocprofv3 FETCH_SIZE reports for the access widths this backend
// uses, on a known byte count (MI355X_MICROARCH.md §HBM: "FETCH_SIZE reports exactly 1/2 of
// the bytes of a wide coalesced streaming read ... other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").
//
// Each kernel reads every byte of a 1 GiB buffer once (4x the 256 MiB Infinity Cache, so the
// counters see memory-side traffic) and writes one dword per workgroup:
//   k_x16   16 B per lane, coalesced (the guide's calibrated case)
//   k_x4    4 B per lane, coalesced (k_inter window rows, k_lf / k_cdef pixel loads)
//   k_x1    1 B per lane, coalesced
//   k_line4 one dword per 64-B segment, i.e. the other 60 B of every segment unread (the
//           byte-granular window rows of random motion: whole lines fetched for a few bytes)
// Run: rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/_build/fetch_calib
// and divide each kernel's FETCH_SIZE (KB) by the bytes its lines span (printed).
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr size_t kBytes = (size_t)1 << 30;

__global__ __launch_bounds__(256) void k_x16(const uint4* __restrict__ p, uint32_t* out, size_t n16)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;  // keeps the loads; never true for the fill
}
__global__ __launch_bounds__(256) void k_x4(const uint32_t* __restrict__ p, uint32_t* out, size_t n4)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) acc ^= p[i];
    if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}
__global__ __launch_bounds__(256) void k_x1(const uint8_t* __restrict__ p, uint32_t* out, size_t n)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc += p[i];
    if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}
__global__ __launch_bounds__(256) void k_line4(const uint32_t* __restrict__ p, uint32_t* out, size_t nLines)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < nLines; i += (size_t)gridDim.x * 256) acc ^= p[i * 16];
    if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}

int main()
{
    void* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 4 << 20) != hipSuccess) return 1;
    (void)hipMemset(buf, 0x11, kBytes);
    (void)hipDeviceSynchronize();
    const int grid = 256 * 16;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_x16, dim3(grid), dim3(256), 0, 0, (const uint4*)buf, out, kBytes / 16);
        hipLaunchKernelGGL(k_x4, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, out, kBytes / 4);
        hipLaunchKernelGGL(k_x1, dim3(grid), dim3(256), 0, 0, (const uint8_t*)buf, out, kBytes);
        hipLaunchKernelGGL(k_line4, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, out, kBytes / 64);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"bytes_spanned\": %zu, \"bytes_loaded\": {\"k_x16\": %zu, \"k_x4\": %zu, \"k_x1\": %zu, \"k_line4\": %zu}}\n",
           kBytes, kBytes, kBytes, kBytes, kBytes / 16);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
