// Probe: is the hardware v_exp_f32 (__builtin_amdgcn_exp2f) correctly rounded on x in [-lim, 0]?
// Compares it with exp2 evaluated in double and rounded to float, over EVERY float in the range,
// and reports the mismatches (and how close the double result was to a float rounding boundary).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>

__global__ void probe(uint32_t lo, uint32_t n, unsigned long long* cnt, uint32_t* samples, int max_samples) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t stride = gridDim.x * blockDim.x;
  unsigned long long bad = 0, near = 0;
  for (; i < n; i += stride) {
    uint32_t bits = lo + i;
    float x = __uint_as_float(bits);
    float hw = __builtin_amdgcn_exp2f(x);
    double d = exp2((double)x);
    float cr = (float)d;
    // distance of d from the float rounding boundary (in units of the float ulp)
    float other = nextafterf(cr, (d > (double)cr) ? 2.0f : -2.0f);
    double mid = 0.5 * ((double)cr + (double)other);
    double rel = fabs(d - mid) / fabs((double)other - (double)cr);
    if (rel < 1e-6) near++;
    if (__float_as_uint(hw) != __float_as_uint(cr)) {
      unsigned long long k = atomicAdd(&cnt[0], 1ull);
      if (k < (unsigned long long)max_samples) {
        samples[3 * k] = bits;
        samples[3 * k + 1] = __float_as_uint(hw);
        samples[3 * k + 2] = __float_as_uint(cr);
      }
    }
  }
  atomicAdd(&cnt[1], near);
  (void)bad;
}

int main(int argc, char** argv) {
  float lim = argc > 1 ? atof(argv[1]) : 8.0f;
  uint32_t lo = 0x80000000u;                 // -0.0
  uint32_t hi = *(uint32_t*)&lim | 0x80000000u;  // -lim
  uint32_t n = hi - lo + 1;
  unsigned long long* cnt;
  uint32_t* samples;
  const int MS = 64;
  hipMalloc(&cnt, 16);
  hipMemset(cnt, 0, 16);
  hipMalloc(&samples, MS * 12);
  probe<<<8192, 256>>>(lo, n, cnt, samples, MS);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
  unsigned long long h[2];
  uint32_t s[MS * 3];
  hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost);
  hipMemcpy(s, samples, sizeof(s), hipMemcpyDeviceToHost);
  printf("range [-%g, 0]: %u floats, mismatches vs correctly-rounded exp2: %llu, near-boundary: %llu\n", lim, n,
         h[0], h[1]);
  for (int k = 0; k < (int)(h[0] < MS ? h[0] : MS); k++) {
    float x = *(float*)&s[3 * k], a = *(float*)&s[3 * k + 1], b = *(float*)&s[3 * k + 2];
    printf("  x=%.9g (0x%08x) hw=%.9g (0x%08x) cr=%.9g (0x%08x) dulp=%d\n", x, s[3 * k], a, s[3 * k + 1], b,
           s[3 * k + 2], (int)(s[3 * k + 1] - s[3 * k + 2]));
  }
  return 0;
}
