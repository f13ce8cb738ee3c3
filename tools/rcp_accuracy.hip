// rcp_accuracy.hip -- diagnostic (not part of the product): ulp error of
// v_rcp_f64 (__builtin_amdgcn_rcp on double) against the correctly rounded
// 1/d, over d in [1, 2^64] (the divisors div_fast sees) and (0.5, 4).
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <string.h>

__global__ void k(const double *d, long long *ulp, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double y = __builtin_amdgcn_rcp(d[i]);
  const double e = 1.0 / d[i];
  long long a, b;
  memcpy(&a, &y, 8);
  memcpy(&b, &e, 8);
  ulp[i] = a > b ? a - b : b - a;
}

int main() {
  const int n = 1 << 22;
  double *h = new double[n];
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double u = (double)(s >> 11) * (1.0 / 9007199254740992.0);
    h[i] = i < n / 2 ? 1.0 + u * 63.0 : 0.5 + u * 3.5;  // [1, 64) and (0.5, 4)
    if (i % 4 == 0 && i < n / 2) h[i] = ldexp(1.0 + u, (int)(s % 64));  // [1, 2^64]
  }
  double *d;
  long long *ulp;
  hipMalloc(&d, n * 8);
  hipMalloc(&ulp, n * 8);
  hipMemcpy(d, h, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, d, ulp, n);
  long long *hu = new long long[n];
  hipMemcpy(hu, ulp, n * 8, hipMemcpyDeviceToHost);
  long long hist[4] = {0, 0, 0, 0}, mx = 0;
  for (int i = 0; i < n; ++i) {
    hist[hu[i] < 3 ? hu[i] : 3]++;
    if (hu[i] > mx) mx = hu[i];
  }
  printf("v_rcp_f64 vs 1/d over %d samples: exact %lld, 1 ulp %lld, 2 ulp %lld, >2 ulp %lld, max %lld\n",
         n, hist[0], hist[1], hist[2], hist[3], mx);
  return 0;
}
