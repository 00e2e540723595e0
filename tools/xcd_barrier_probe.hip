// Cost of a barrier among the workgroups of ONE XCD inside a launch (VERDICT
// r03 item 3: a persistent single-XCD kernel for the 4 k - 130 k-row AMG
// levels, whose phases would be separated by such barriers instead of kernel
// boundaries).  A grid of 256 workgroups is launched; the 32 with
// blockIdx % 8 == 0 (one XCD under round-robin dispatch) run P phases, the
// others exit.  Each phase: every thread stores one float of a 32 x 256 vector
// slice, then the barrier, then every thread reads a value another workgroup
// stored (checked).  Barrier forms (the memory-model rules of
// cdna_hip_programming.md Guideline 16):
//   0 release: plain stores, agent-scope release fence, relaxed atomic arrive,
//     relaxed polls with s_sleep, agent-scope acquire, plain loads
//   1 write-through: payload stores by agent-scope relaxed atomics (sc1, no
//     release fence needed), drain, arrive, poll, agent-scope acquire
//   2 write-through + sc1 loads: as 1, payload read by agent-scope relaxed
//     atomic loads (bypass L1), no acquire fence
// Per-phase cost = (T(P) - T(0)) / P, host-paired over a launch, best of 7.
// Every poll is bounded (2^22 spins): a timeout sets a flag and the workgroup
// leaves, so the grid always drains.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

constexpr int kWG = 32, kT = 256;

__device__ __forceinline__ bool arrive_wait(unsigned* cnt, unsigned target, unsigned* tmo) {
  // one lane per workgroup; the caller holds the workgroup at __syncthreads()
  __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (unsigned spins = 0; spins < (1u << 22); ++spins) {
    if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return false;
}

template <int FORM>
__global__ void __launch_bounds__(kT) k_probe(float* vec, unsigned* cnt, unsigned* tmo, unsigned* bad, int P) {
  if (blockIdx.x % 8 != 0) return;
  const int w = blockIdx.x / 8;  // 0..31
  const int t = threadIdx.x;
  __shared__ int ok;
  for (int ph = 0; ph < P; ++ph) {
    float* cur = vec + (size_t)(ph & 1) * kWG * kT;
    const float val = (float)(ph * 1000 + w * 7 + t);
    if (FORM == 0) {
      cur[w * kT + t] = val;
    } else {
      __hip_atomic_store(reinterpret_cast<unsigned*>(cur) + w * kT + t, __float_as_uint(val), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (FORM == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (t == 0) ok = arrive_wait(cnt, (unsigned)(kWG * (ph + 1)), tmo) ? 1 : 0;
    __syncthreads();
    if (!ok) return;
    if (FORM != 2) {
      if (t == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __syncthreads();
    }
    const int ow = (w + 1 + ph) % kWG;
    float got;
    if (FORM == 2)
      got = __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(cur) + ow * kT + t, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT));
    else
      got = cur[ow * kT + t];
    if (got != (float)(ph * 1000 + ow * 7 + t)) atomicAdd(bad, 1u);
  }
}

int main() {
  float* vec;
  unsigned *cnt, *flags;
  CK(hipMalloc(&vec, 2 * kWG * kT * sizeof(float)));
  CK(hipMalloc(&flags, 64));
  cnt = flags;
  unsigned* tmo = flags + 4;
  unsigned* bad = flags + 8;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  static const char* names[] = {"release+acquire", "sc1-store+acquire", "sc1-store+sc1-load"};
  for (int form = 0; form < 3; ++form) {
    double base = 0.0;
    for (int P : {0, 100, 1000}) {
      float best = 1e30f;
      unsigned h[16] = {};
      for (int r = 0; r < 7; ++r) {
        CK(hipMemset(flags, 0, 64));
        CK(hipEventRecord(e0));
        if (form == 0)
          hipLaunchKernelGGL(k_probe<0>, dim3(256), dim3(kT), 0, 0, vec, cnt, tmo, bad, P);
        else if (form == 1)
          hipLaunchKernelGGL(k_probe<1>, dim3(256), dim3(kT), 0, 0, vec, cnt, tmo, bad, P);
        else
          hipLaunchKernelGGL(k_probe<2>, dim3(256), dim3(kT), 0, 0, vec, cnt, tmo, bad, P);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
        CK(hipMemcpy(h, flags, 64, hipMemcpyDeviceToHost));
        if (h[4] || h[8]) break;
      }
      if (P == 0) base = best;
      std::printf("form %-20s P=%5d  launch %.2f us  per phase %.3f us  timeout=%u wrong=%u\n", names[form], P,
                  best * 1e3, P ? (best - base) * 1e3 / P : 0.0, h[4], h[8]);
      if (h[4]) return 2;
    }
  }
  return 0;
}
