// probe_lasterror.hip -- does hipStreamQuery's hipErrorNotReady stay in the
// thread's last error (hipGetLastError after a later, successful launch)?
//   hipcc --offload-arch=gfx950 -O2 -o ab/probe_lasterror scripts/probe_lasterror.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void spin(unsigned long long cycles) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < cycles) {
    }
}
__global__ void nop() {}

int main() {
    hipStream_t a, b;
    (void)hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, 2000000ull);  // 20 ms
    const hipError_t q = hipStreamQuery(a);
    hipLaunchKernelGGL(nop, dim3(1), dim3(64), 0, b);
    const hipError_t g1 = hipGetLastError();
    const hipError_t g2 = hipGetLastError();
    const hipError_t q2 = hipStreamQuery(a);
    const hipError_t p1 = hipPeekAtLastError();
    (void)hipStreamSynchronize(a);
    (void)hipStreamSynchronize(b);
    printf("{\"query\": \"%s\", \"last_after_launch\": \"%s\", \"last_again\": \"%s\", \"query2\": \"%s\", \"peek_after_query2\": \"%s\"}\n",
           hipGetErrorName(q), hipGetErrorName(g1), hipGetErrorName(g2), hipGetErrorName(q2), hipGetErrorName(p1));
    return 0;
}
