// Shader-clock probe (tools only, not part of libmec_hip.so): one wave that samples
// (s_memtime, s_memrealtime) every ~4 us while other work runs, so the host can read the clock
// the chip holds under that load (MI355X_MICROARCH.md, DVFS give-back: s_memtime counts shader
// cycles, s_memrealtime 100 MHz). Output stored by vector stores, one 16-B pair per sample.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/clock_probe.hip -o build/clock_probe.so
#include <hip/hip_runtime.h>

__global__ void clock_probe_kernel(unsigned long long* out, int n, const volatile int* stop) {
  if (threadIdx.x != 0) return;
  for (int i = 0; i < n; ++i) {
    const unsigned long long c = __builtin_amdgcn_s_memtime();
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    out[2 * i + threadIdx.x] = c;
    out[2 * i + 1 + threadIdx.x] = r;
    if (*stop) {
      out[2 * i + 2 + threadIdx.x] = 0;
      return;
    }
    __builtin_amdgcn_s_sleep(127);  // ~8k cycles between samples
  }
}

extern "C" int clock_probe_launch(void* out, int n, const int* stop, void* stream) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     reinterpret_cast<unsigned long long*>(out), n, stop);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
