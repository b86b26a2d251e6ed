// Does hipMemcpyAsync (host -> device, pinned source) return before the
// transfer is done?  Per variant: host time inside the call(s), time to
// completion, GB/s.  Variants: pinned allocation flags x copy API x size.
// Build: hipcc --offload-arch=gfx950 -O2 memcpy_async.cpp -o memcpy_async
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t big = 80ull << 20;  // one 131k-signature chunk of config 2
  void* d = nullptr;
  CK(hipMalloc(&d, 4 * big));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct Alloc { const char* name; unsigned flags; bool reg; };
  const Alloc allocs[] = {{"hipHostMalloc(Default)", hipHostMallocDefault, false},
                          {"hipHostMalloc(Portable|Mapped)", hipHostMallocPortable | hipHostMallocMapped, false},
                          {"hipHostMalloc(NonCoherent)", hipHostMallocNonCoherent, false},
                          {"malloc+hipHostRegister(Default)", 0, true}};
  for (const auto& al : allocs) {
    void* h = nullptr;
    if (al.reg) {
      h = aligned_alloc(4096, 4 * big);
      CK(hipHostRegister(h, 4 * big, hipHostRegisterDefault));
    } else {
      CK(hipHostMalloc(&h, 4 * big, al.flags));
    }
    std::memset(h, 1, 4 * big);
    for (size_t sz : {big / 64, big / 8, big, 4 * big}) {
      for (int api = 0; api < 2; ++api) {
        CK(hipStreamSynchronize(s));
        double best_call = 1e30, best_total = 1e30;
        for (int rep = 0; rep < 4; ++rep) {
          const double t0 = now_us();
          if (api == 0) CK(hipMemcpyAsync(d, h, sz, hipMemcpyHostToDevice, s));
          else CK(hipMemcpyAsync(d, h, sz, hipMemcpyDefault, s));
          const double t1 = now_us();
          CK(hipStreamSynchronize(s));
          const double t2 = now_us();
          if (rep) {
            best_call = std::min(best_call, t1 - t0);
            best_total = std::min(best_total, t2 - t0);
          }
        }
        std::printf("%-34s %-8s %8.1f MB  call %8.1f us  done %8.1f us  %6.1f GB/s\n", al.name,
                    api ? "Default" : "HtoD", sz / 1e6, best_call, best_total, sz / best_total / 1e3);
      }
    }
    // two copies back to back: does the second call wait for the first transfer?
    CK(hipStreamSynchronize(s));
    const double t0 = now_us();
    CK(hipMemcpyAsync(d, h, big, hipMemcpyHostToDevice, s));
    const double t1 = now_us();
    CK(hipMemcpyAsync((char*)d + big, (char*)h + big, big, hipMemcpyHostToDevice, s));
    const double t2 = now_us();
    CK(hipStreamSynchronize(s));
    const double t3 = now_us();
    std::printf("%-34s two 84 MB copies: call1 %.1f us, call2 %.1f us, done %.1f us\n", al.name, t1 - t0, t2 - t1, t3 - t0);
    if (al.reg) {
      CK(hipHostUnregister(h));
      free(h);
    } else {
      CK(hipHostFree(h));
    }
  }
  return 0;
}
