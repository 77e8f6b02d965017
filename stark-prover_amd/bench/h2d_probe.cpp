// Dev probe: where the host-input commit's extra time goes (BASELINE
// `pcie_inclusive`): the canonical check over d coefficients, a pageable
// hipMemcpy, a pinned one, and host staging into pinned memory with 1..8
// threads.  hipcc -O3 -std=c++17 h2d_probe.cpp -o h2d_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
static uint32_t maxscan(const uint32_t* v, size_t n) {
    uint32_t mx = 0;
    for (size_t j = 0; j < n; j++) mx = v[j] > mx ? v[j] : mx;
    return mx;
}
static uint32_t copymax(const uint32_t* s, uint32_t* d, size_t n) {
    uint32_t mx = 0;
    for (size_t j = 0; j < n; j++) { const uint32_t v = s[j]; d[j] = v; mx = v > mx ? v : mx; }
    return mx;
}
int main() {
    const size_t n = (size_t)1 << 21, bytes = n * 4;
    std::vector<uint32_t> host(n);
    for (size_t i = 0; i < n; i++) host[i] = (uint32_t)(i * 2654435761u) % 3221225473u;
    uint32_t *pin, *dev;
    CK(hipHostMalloc((void**)&pin, bytes));
    CK(hipMalloc((void**)&dev, bytes));
    hipStream_t s; CK(hipStreamCreate(&s));
    volatile uint32_t sink = 0;
    for (int rep = 0; rep < 3; rep++) {
        double t0 = now(); sink += maxscan(host.data(), n); double t1 = now();
        CK(hipMemcpyAsync(dev, host.data(), bytes, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s)); double t2 = now();
        CK(hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s)); double t3 = now();
        sink += copymax(host.data(), pin, n); double t4 = now();
        printf("rep %d: check %.3f ms  pageable H2D %.3f ms  pinned H2D %.3f ms  copy+max 1 thread %.3f ms\n", rep,
               (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3);
        for (int T : {2, 4, 8}) {
            double a = now();
            std::vector<std::thread> th;
            std::vector<uint32_t> m(T);
            for (int i = 0; i < T; i++) th.emplace_back([&, i] { const size_t c = n / T; m[i] = copymax(host.data() + i * c, pin + i * c, c); });
            for (auto& t : th) t.join();
            double b = now();
            // staged in 4 chunks: copy chunk c (T threads) then DMA it while the next is copied
            const size_t C = 4, cs = n / C;
            for (size_t c = 0; c < C; c++) {
                std::vector<std::thread> t2v;
                for (int i = 0; i < T; i++) t2v.emplace_back([&, i, c] { const size_t q = cs / T; copymax(host.data() + c * cs + i * q, pin + c * cs + i * q, q); });
                for (auto& t : t2v) t.join();
                CK(hipMemcpyAsync(dev + c * cs, pin + c * cs, cs * 4, hipMemcpyHostToDevice, s));
            }
            CK(hipStreamSynchronize(s));
            double e = now();
            printf("   %d threads: copy+max %.3f ms; chunked copy+max+DMA %.3f ms\n", T, (b - a) * 1e3, (e - b) * 1e3);
        }
    }
    printf("sink %u\n", (unsigned)sink);
    return 0;
}
