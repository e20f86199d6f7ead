// cvt_probe: what v_cvt_rpi_i32_f32 and v_cvt_flr_i32_f32 return on this
// GPU (rounding of x + 0.5, saturation, NaN), against host expectations.
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/cvt_probe tools/dbg/cvt_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_probe(const float *x, int *rpi, int *flr, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int a, b;
    __asm__ volatile("v_cvt_rpi_i32_f32 %0, %1" : "=v"(a) : "v"(x[i]));
    __asm__ volatile("v_cvt_flr_i32_f32 %0, %1" : "=v"(b) : "v"(x[i]));
    rpi[i] = a;
    flr[i] = b;
}

static int sat(double v) {
    if (std::isnan(v)) return 0;
    if (v >= 2147483647.0) return 2147483647;
    if (v <= -2147483648.0) return (int)-2147483648LL;
    return (int)v;
}

int main() {
    std::vector<float> x;
    for (int k = -40000; k <= 40000; k += 7)
        for (int d = -3; d <= 3; d++) {
            float v = (float)k + 0.5f; /* a tie and its 3 neighbours on each side */
            for (int j = 0; j < (d < 0 ? -d : d); j++) v = std::nextafter(v, d < 0 ? -1e30f : 1e30f);
            x.push_back(v);
        }
    for (float v = 0.49999f; v < 0.50001f; v = std::nextafter(v, 1.f)) { x.push_back(v); x.push_back(-v); }
    const float sp[] = {0.f, -0.f, 1e10f, -1e10f, 2147483520.f, 2147483648.f, -2147483648.f, -2147483904.f,
                        INFINITY, -INFINITY, NAN, 1.5f, 2.5f, -1.5f, -2.5f, 32767.5f, -32768.5f};
    for (float v : sp) x.push_back(v);
    const int n = (int)x.size();
    float *dx; int *dr, *df;
    hipMalloc(&dx, n * 4); hipMalloc(&dr, n * 4); hipMalloc(&df, n * 4);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dr, df, n);
    std::vector<int> r(n), f(n);
    hipMemcpy(r.data(), dr, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(f.data(), df, n * 4, hipMemcpyDeviceToHost);
    int bad_exact = 0, bad_f32add = 0, bad_flr = 0;
    for (int i = 0; i < n; i++) {
        const int e_exact = sat(std::floor((double)x[i] + 0.5));       // floor of the exact sum
        const int e_f32 = sat(std::floor((double)(float)(x[i] + 0.5f))); // floor of the f32 sum
        const int e_flr = sat(std::floor((double)x[i]));
        bad_exact += r[i] != e_exact;
        bad_f32add += r[i] != e_f32;
        bad_flr += f[i] != e_flr;
        if ((r[i] != e_exact || r[i] != e_f32) && bad_exact + bad_f32add < 12)
            printf("x=%.9g rpi=%d exact=%d f32add=%d\n", x[i], r[i], e_exact, e_f32);
    }
    for (float v : sp) {
        int i = 0;
        while (memcmp(&x[i], &v, 4)) i++;
        printf("x=%g rpi=%d flr=%d\n", v, r[i], f[i]);
    }
    printf("n=%d rpi!=floor(exact x+0.5): %d  rpi!=floor(f32(x+0.5)): %d  flr!=floor(x): %d\n", n, bad_exact, bad_f32add,
           bad_flr);
    return 0;
}
