// Latency probe for the dataflow kernels' per-item costs on gfx950 (one wave unless noted):
// dependent chains of scalar loads, vector loads, LDS loads; a vector load issued behind
// N outstanding stores; s_memrealtime back to back; workgroup barriers (4 waves).
// Build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/latency_probe tools/latency_probe.hip
// Prints ns per operation (s_memrealtime: 100 MHz).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REPS 256
typedef __attribute__((address_space(4))) const uint32_t* cptr;

__device__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

extern "C" __global__ void k_probe(const uint32_t* chain, uint32_t* scratch, uint64_t* out)
{
    __shared__ uint32_t lds[1024];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += blockDim.x) lds[i] = (i * 17 + 1) & 1023;
    __syncthreads();
    if (threadIdx.x >= 64) {  // waves 1..3 only join the barrier test
        for (int r = 0; r < REPS; r++) __syncthreads();
        return;
    }
    uint64_t t0, t1;
    uint32_t idx = 0, acc = 0;
    // 1: scalar load chain (K$ after the first pass)
    for (int pass = 0; pass < 2; pass++) {
        idx = 0;
        t0 = now();
        for (int r = 0; r < REPS; r++) idx = *(cptr)(uintptr_t)(chain + idx);
        t1 = now();
    }
    acc += idx;
    if (lane == 0) out[0] = t1 - t0;
    // 2: vector load chain (per-lane index = same value: L1 / L2 hits)
    for (int pass = 0; pass < 2; pass++) {
        uint32_t v = lane & 0;
        t0 = now();
        for (int r = 0; r < REPS; r++) v = __builtin_nontemporal_load(chain + v + (lane & 0));
        t1 = now();
        acc += v;
    }
    if (lane == 0) out[1] = t1 - t0;
    // 3: LDS chain
    {
        uint32_t v = lane & 0;
        t0 = now();
        for (int r = 0; r < REPS; r++) v = lds[v];
        t1 = now();
        acc += v;
    }
    if (lane == 0) out[2] = t1 - t0;
    // 4: s_memrealtime back to back
    {
        t0 = now();
        uint64_t x = 0;
        for (int r = 0; r < REPS; r++) x += now();
        t1 = now();
        acc += (uint32_t)x;
    }
    if (lane == 0) out[3] = t1 - t0;
    // 5: a store (plain) then a dependent vector load of another line, repeated
    {
        uint32_t v = 0;
        t0 = now();
        for (int r = 0; r < REPS; r++) {
            scratch[(r & 63) * 64 + lane] = v + r;
            v = __builtin_nontemporal_load(chain + (v & 7) + (lane & 0));
        }
        t1 = now();
        acc += v;
    }
    if (lane == 0) out[4] = t1 - t0;
    // 6: agent-scope atomic store (sc1) then a dependent vector load
    {
        uint32_t v = 0;
        t0 = now();
        for (int r = 0; r < REPS; r++) {
            __hip_atomic_store(scratch + 8192 + (r & 63) * 64 + lane, v + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v = __builtin_nontemporal_load(chain + (v & 7) + (lane & 0));
        }
        t1 = now();
        acc += v;
    }
    if (lane == 0) out[5] = t1 - t0;
    // 7: a store then a dependent SCALAR load chain step
    {
        uint32_t s = 0;
        t0 = now();
        for (int r = 0; r < REPS; r++) {
            scratch[16384 + (r & 63) * 64 + lane] = s + r;
            s = *(cptr)(uintptr_t)(chain + (s & 7));
        }
        t1 = now();
        acc += s;
    }
    if (lane == 0) out[6] = t1 - t0;
    // 8: agent-scope atomic load chain (sc1: bypasses L1)
    {
        uint32_t v = 0;
        t0 = now();
        for (int r = 0; r < REPS; r++) v = __hip_atomic_load(chain + (v & 7) + (lane & 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t1 = now();
        acc += v;
    }
    if (lane == 0) out[7] = t1 - t0;
    // 9: barrier (4 waves)
    t0 = now();
    for (int r = 0; r < REPS; r++) __syncthreads();
    t1 = now();
    if (lane == 0) out[8] = t1 - t0;
    if (acc == 0x12345678) out[15] = acc;
}

int main()
{
    uint32_t h[1024];
    for (int i = 0; i < 1024; i++) h[i] = (i * 7 + 3) & 7;  // chain stays within the first 8 words
    uint32_t *chain, *scratch;
    uint64_t* out;
    hipMalloc(&chain, sizeof(h));
    hipMalloc(&scratch, 4 << 20);
    hipMalloc(&out, 16 * 8);
    hipMemcpy(chain, h, sizeof(h), hipMemcpyHostToDevice);
    const char* names[] = {"s_load chain", "vector load chain", "LDS load chain", "s_memrealtime", "plain store + vector load",
        "sc1 store + vector load", "plain store + s_load", "sc1 load chain", "barrier (4 waves)"};
    for (int rep = 0; rep < 3; rep++) {
        hipMemset(out, 0, 16 * 8);
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(256), 0, 0, chain, scratch, out);
        uint64_t o[16];
        if (hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost) != hipSuccess) {
            printf("failed\n");
            return 1;
        }
        for (int i = 0; i < 9; i++) printf("%-28s %8.1f ns/op\n", names[i], o[i] * 10.0 / REPS);
        printf("\n");
    }
    return 0;
}
