// Kernel-boundary cost probe (gfx950): per-kernel time inside a captured hipGraph for
//   empty 1-block kernels, 250x512-thread kernels holding ~100 KB LDS, the same writing an
//   11 MB slab (the fused train kernel's gradient partials), and a persistent kernel that
//   replaces two boundaries with two grid barriers (agent-scope atomics).
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/overhead_probe.hip -o /tmp/overhead_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

__global__ void k_empty() {}

__global__ void k_lds(float* out) {
    extern __shared__ float lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (lds[(threadIdx.x + 1) % blockDim.x] < 0.f) out[0] = 1.f;
}

__global__ void k_slab(float* slab, int per_block) {
    extern __shared__ float lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    float* s = slab + (size_t)blockIdx.x * per_block;
    for (int i = threadIdx.x; i < per_block; i += blockDim.x) s[i] = lds[i % blockDim.x];
}

// grid barrier: counter incremented by every block, spin until it reaches target
__device__ void grid_sync(unsigned* ctr, unsigned target) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // bounded spin: a grid that is not fully resident gives up instead of hanging
        for (int it = 0; it < 2000000 && __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++it)
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

__global__ void k_persist(float* slab, int per_block, unsigned* ctr, unsigned base) {
    extern __shared__ float lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    float* s = slab + (size_t)blockIdx.x * per_block;
    for (int i = threadIdx.x; i < per_block; i += blockDim.x) s[i] = lds[i % blockDim.x];
    grid_sync(ctr, base + gridDim.x);
    grid_sync(ctr, base + 2 * gridDim.x);
}

int main() {
    const int B = 250, T = 512, per_block = 11352, N = 200;
    const size_t lds = 100 * 1024;
    float *slab, *out;
    unsigned* ctr;
    CK(hipMalloc(&slab, (size_t)B * 2 * per_block * 4));
    CK(hipMalloc(&out, 4));
    CK(hipMalloc(&ctr, 4));
    CK(hipFuncSetAttribute((const void*)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)k_slab, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)k_persist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_graph = [&](const char* name, auto&& body) -> int {
        hipGraph_t g; hipGraphExec_t x;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < N; ++i) body(i);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
        CK(hipMemsetAsync(ctr, 0, 4, s));
        CK(hipGraphLaunch(x, s));
        CK(hipStreamSynchronize(s));
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipMemsetAsync(ctr, 0, 4, s));
            CK(hipEventRecord(e0, s));
            CK(hipGraphLaunch(x, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%-44s %8.2f us per launch\n", name, best * 1e3f / N);
        CK(hipGraphExecDestroy(x)); CK(hipGraphDestroy(g));
        return 0;
    };
    time_graph("empty <<<1,64>>>", [&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); });
    time_graph("empty <<<250,512>>>", [&](int) { hipLaunchKernelGGL(k_empty, dim3(B), dim3(T), 0, s); });
    time_graph("lds 100KB <<<250,512>>>", [&](int) { hipLaunchKernelGGL(k_lds, dim3(B), dim3(T), lds, s, out); });
    time_graph("lds 100KB <<<500,512>>>", [&](int) { hipLaunchKernelGGL(k_lds, dim3(2 * B), dim3(T), lds / 2, s, out); });
    time_graph("slab 11MB <<<250,512>>>", [&](int) { hipLaunchKernelGGL(k_slab, dim3(B), dim3(T), lds, s, slab, per_block); });
    time_graph("slab 1.1MB <<<250,512>>>", [&](int) { hipLaunchKernelGGL(k_slab, dim3(B), dim3(T), lds, s, slab, per_block / 10); });
    time_graph("3 x slab-kernel chain (per chain)", [&](int) {
        hipLaunchKernelGGL(k_slab, dim3(B), dim3(T), lds, s, slab, per_block);
        hipLaunchKernelGGL(k_lds, dim3(B), dim3(T), lds, s, out);
        hipLaunchKernelGGL(k_lds, dim3(B), dim3(T), lds, s, out);
    });
    time_graph("persistent slab + 2 grid barriers", [&](int i) {
        hipLaunchKernelGGL(k_persist, dim3(B), dim3(T), lds, s, slab, per_block, ctr, (unsigned)(2 * B * i));
    });
    return 0;
}
