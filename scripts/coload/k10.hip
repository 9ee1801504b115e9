#include <hip/hip_runtime.h>
extern "C" __global__ void k0(float* p, int n) { int j = blockIdx.x * blockDim.x + threadIdx.x; if (j < n) p[j] = p[j] * 0.5f + 0; }
extern "C" __global__ void k1(float* p, int n) { int j = blockIdx.x * blockDim.x + threadIdx.x; if (j < n) p[j] = p[j] * 1.5f + 1; }
extern "C" __global__ void k2(float* p, int n) { int j = blockIdx.x * blockDim.x + threadIdx.x; if (j < n) p[j] = p[j] * 2.5f + 2; }
extern "C" __global__ void k3(float* p, int n) { int j = blockIdx.x * blockDim.x + threadIdx.x; if (j < n) p[j] = p[j] * 3.5f + 3; }
extern "C" __global__ void k4(float* p, int n) { int j = blockIdx.x * blockDim.x + threadIdx.x; if (j < n) p[j] = p[j] * 4.5f + 4; }
extern "C" __global__ void k5(float* p, int n) { int j = blockIdx.x * blockDim.x + threadIdx.x; if (j < n) p[j] = p[j] * 5.5f + 5; }
extern "C" __global__ void k6(float* p, int n) { int j = blockIdx.x * blockDim.x + threadIdx.x; if (j < n) p[j] = p[j] * 6.5f + 6; }
extern "C" __global__ void k7(float* p, int n) { int j = blockIdx.x * blockDim.x + threadIdx.x; if (j < n) p[j] = p[j] * 7.5f + 7; }
extern "C" __global__ void k8(float* p, int n) { int j = blockIdx.x * blockDim.x + threadIdx.x; if (j < n) p[j] = p[j] * 8.5f + 8; }
extern "C" __global__ void k9(float* p, int n) { int j = blockIdx.x * blockDim.x + threadIdx.x; if (j < n) p[j] = p[j] * 9.5f + 9; }
