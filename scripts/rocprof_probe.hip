// Minimal HIP program to check whether rocprofv3 kernel tracing works on the box.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void axpy(float* y, const float* x, float a, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] += a * x[i];
}
int main() {
    const int n = 1 << 20;
    float *x, *y;
    if (hipMalloc(&x, n * 4) != hipSuccess || hipMalloc(&y, n * 4) != hipSuccess) return 1;
    (void)hipMemset(x, 0, n * 4);
    (void)hipMemset(y, 0, n * 4);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(axpy, dim3(n / 256), dim3(256), 0, 0, y, x, 2.f, n);
    (void)hipDeviceSynchronize();
    printf("probe ok\n");
    return 0;
}
