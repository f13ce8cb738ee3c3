// Host <-> device round trip (diagnostic for the window server's round
// latency): one lane spins on a flag, answers each new value through a word
// in host-mapped memory, and the host posts the next value once it sees the
// answer.  The flag lives either in host-mapped memory (what the window
// server polls today: every poll is a PCIe read) or in fine-grained device
// memory the host writes through the BAR (the poll stays in HBM / L2).
//   hipcc --offload-arch=gfx950 -O2 tools/pcie_pingpong.hip -o tools/pcie_pingpong
#include <hip/hip_runtime.h>
#include <x86intrin.h>

#include <chrono>
#include <csignal>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                    \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__device__ __forceinline__ uint64_t ticks() { return __builtin_amdgcn_s_memrealtime(); }

// reply[0]: answers; reply[1]: ticks spent spinning; reply[2]: polls
__global__ void pingpong(const uint64_t *flag, uint64_t *reply, int n, uint64_t deadline) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = ticks();
  uint64_t polls = 0;
  for (int i = 1; i <= n; ++i) {
    for (;;) {
      const uint64_t v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      ++polls;
      if (v == (uint64_t)i) break;
      if (ticks() - t0 > deadline) {
        __hip_atomic_store(reply, ~0ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
    }
    __hip_atomic_store(reply, (uint64_t)i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __hip_atomic_store(reply + 2, polls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(reply + 1, ticks() - t0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One wave reads K keys (8-byte words) rep times; out[m]: ticks per read of
// all K.  mode 0: 8-byte system-scope loads, every lane's loads in flight
// together (K <= 1024); 1: 16-byte volatile loads, all in flight; 2: one
// 8-byte load per lane at a time.
template <int MODE>
__global__ void keyread(const uint64_t *p, int K, int rep, uint64_t *out) {
  const int lane = threadIdx.x;
  uint64_t acc = 0, best = ~0ull, sum = 0;
  for (int r = 0; r < rep; ++r) {
    const uint64_t t0 = ticks();
    if (MODE == 0) {
      uint64_t v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        v[j] = 64 * j + lane < K ? __hip_atomic_load(p + 64 * j + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc += v[j];
    } else if (MODE == 1) {
      typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
      const volatile u2 *q = (const volatile u2 *)p;
      u2 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 64 * j + lane;
        v[j] = 2 * i < K ? q[i] : u2{0, 0};
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += v[j].x + v[j].y;
    } else {
      for (int j = 0; 64 * j < K; ++j)
        acc += __hip_atomic_load(p + 64 * j + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + (acc & 1);
    }
    acc = __builtin_amdgcn_readfirstlane((int)acc);  // wait for every load
    const uint64_t dt = ticks() - t0;
    sum += dt;
    best = dt < best ? dt : best;
  }
  if (lane == 0) {
    out[0] = sum / rep;
    out[1] = best;
    out[2] = acc;
  }
}

static void keyreads(const char *where, const uint64_t *p, uint64_t *out) {
  const int Ks[] = {64, 256, 512, 1024};
  for (int K : Ks) {
    double t[3][2];
    for (int m = 0; m < 3; ++m) {
      if (m == 1 && K > 1024) continue;
      if (m == 0) hipLaunchKernelGGL(keyread<0>, dim3(1), dim3(64), 0, 0, p, K, 50, out);
      if (m == 1) hipLaunchKernelGGL(keyread<1>, dim3(1), dim3(64), 0, 0, p, K, 50, out);
      if (m == 2) hipLaunchKernelGGL(keyread<2>, dim3(1), dim3(64), 0, 0, p, K, 50, out);
      CHECK(hipDeviceSynchronize());
      t[m][0] = out[0] / 100.0;
      t[m][1] = out[1] / 100.0;
    }
    std::printf("%s K=%5d: 8B in flight %6.2f us (best %6.2f), 16B in flight %6.2f (%6.2f), "
                "8B one per lane at a time %6.2f (%6.2f)\n",
                where, K, t[0][0], t[0][1], t[1][0], t[1][1], t[2][0], t[2][1]);
  }
}

// The window server's poll: lane 0 reads the round word, lanes 1..63 key
// slots 0..62, one load each; on a new round, stale slots (tag < round) are
// read again until fresh.  hist[r]: rounds that needed r re-reads (r <= 3:
// 3 or more).  The host writes the 63 keys, then the round word; the round
// word sits 256 bytes before the keys (the server's layout) or in the word
// right before them (the same 64-byte line as keys 0..6).
__global__ void pollkeys(const uint64_t *round, const uint64_t *keys, uint64_t *reply, int n,
                         uint64_t deadline) {
  const int lane = threadIdx.x;
  const uint64_t t0 = ticks();
  uint64_t hist[4] = {0, 0, 0, 0}, tre = 0;
  for (int i = 1; i <= n; ++i) {
    uint64_t v;
    for (;;) {
      v = __hip_atomic_load(lane == 0 ? round : keys + lane - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (__builtin_amdgcn_readfirstlane((int)v) == i) break;
      if (ticks() - t0 > deadline) {
        if (lane == 0) __hip_atomic_store(reply, ~0ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
    }
    const uint64_t ts = ticks();
    int r = 0;
    while (__ballot(lane > 0 && v < (uint64_t)i)) {
      if (lane > 0 && v < (uint64_t)i)
        v = __hip_atomic_load(keys + lane - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ++r;
    }
    tre += ticks() - ts;
    hist[r < 3 ? r : 3] += 1;
    if (lane == 0) __hip_atomic_store(reply, (uint64_t)i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (lane == 0) {
    for (int j = 0; j < 4; ++j) reply[4 + j] = hist[j];
    reply[8] = tre;
  }
}

static void pollkeys_run(const char *name, uint64_t *h_round, uint64_t *h_keys, const uint64_t *d_round,
                         const uint64_t *d_keys, uint64_t *reply, int n) {
  *(volatile uint64_t *)h_round = 0;
  for (int j = 0; j < 63; ++j) h_keys[j] = 0;
  reply[0] = 0;
  hipLaunchKernelGGL(pollkeys, dim3(1), dim3(64), 0, 0, d_round, d_keys, reply, n, (uint64_t)100000000);
  CHECK(hipGetLastError());
  usleep(20000);
  const auto t0 = std::chrono::steady_clock::now();
  bool ok = true;
  for (int i = 1; i <= n && ok; ++i) {
    for (int j = 0; j < 63; ++j) __atomic_store_n(h_keys + j, (uint64_t)i, __ATOMIC_RELAXED);
    __atomic_store_n(h_round, (uint64_t)i, __ATOMIC_RELEASE);
    for (;;) {
      const uint64_t v = __atomic_load_n(reply, __ATOMIC_ACQUIRE);
      if (v == (uint64_t)i) break;
      if (v == ~0ull) { ok = false; break; }
    }
  }
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  CHECK(hipDeviceSynchronize());
  if (!ok) { std::printf("%s: the kernel never saw a round\n", name); return; }
  std::printf("%-40s %6.3f us per round; re-reads 0/1/2/3+: %llu %llu %llu %llu; %.2f us re-reading per round\n",
              name, us / n, (unsigned long long)reply[4], (unsigned long long)reply[5],
              (unsigned long long)reply[6], (unsigned long long)reply[7], reply[8] / 100.0 / n);
}

static void on_segv(int) {
  const char m[] = "CPU access to device memory faulted (no large BAR mapping)\n";
  ssize_t r = write(1, m, sizeof m - 1);
  (void)r;
  _exit(3);
}

static double run(const char *name, uint64_t *flag_host_view, const uint64_t *flag_dev_view,
                  uint64_t *reply, int n) {
  __atomic_store_n(flag_host_view, 0ull, __ATOMIC_SEQ_CST);
  _mm_sfence();
  reply[0] = 0;
  reply[1] = 0;
  hipLaunchKernelGGL(pingpong, dim3(1), dim3(64), 0, 0, flag_dev_view, reply, n,
                     (uint64_t)100000000);  // 1 s at 100 MHz
  CHECK(hipGetLastError());
  // let the kernel start before the clock runs
  usleep(20000);
  const auto t0 = std::chrono::steady_clock::now();
  bool ok = true;
  for (int i = 1; i <= n && ok; ++i) {
    __atomic_store_n(flag_host_view, (uint64_t)i, __ATOMIC_SEQ_CST);
    _mm_sfence();
    for (;;) {
      const uint64_t v = __atomic_load_n(reply, __ATOMIC_ACQUIRE);
      if (v == (uint64_t)i) break;
      if (v == ~0ull) { ok = false; break; }
    }
  }
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  CHECK(hipDeviceSynchronize());
  if (!ok) {
    std::printf("%-34s the kernel never saw a posted value\n", name);
    return -1;
  }
  std::printf("%-34s %7.3f us per round trip (%d trips, %.1f polls per trip)\n", name, us / n, n,
              (double)reply[2] / n);
  return us / n;
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
  uint64_t *reply = nullptr, *hflag = nullptr;
  CHECK(hipHostMalloc((void **)&reply, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostMalloc((void **)&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  uint64_t *hflag_dev = nullptr;
  CHECK(hipHostGetDevicePointer((void **)&hflag_dev, hflag, 0));
  run("flag in host memory (PCIe poll)", hflag, hflag_dev, reply, n);
  uint64_t *hkeys = nullptr, *hkeys_dev = nullptr;
  CHECK(hipHostMalloc((void **)&hkeys, 8192 * 8, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostGetDevicePointer((void **)&hkeys_dev, hkeys, 0));
  for (int i = 0; i < 8192; ++i) hkeys[i] = i;
  keyreads("host memory  ", hkeys_dev, reply + 4);
  pollkeys_run("poll: round word 256 B before the keys", hkeys, hkeys + 32, hkeys_dev, hkeys_dev + 32, reply, n);
  pollkeys_run("poll: round word in the keys' line", hkeys + 64, hkeys + 65, hkeys_dev + 64, hkeys_dev + 65, reply, n);

  uint64_t *dflag = nullptr;
  CHECK(hipExtMallocWithFlags((void **)&dflag, 4096, hipDeviceMallocFinegrained));
  hipPointerAttribute_t a{};
  CHECK(hipPointerGetAttributes(&a, dflag));
  std::printf("fine-grained device allocation: type %d device %p host %p\n", (int)a.type,
              a.devicePointer, a.hostPointer);
  std::fflush(stdout);
  std::signal(SIGSEGV, on_segv);
  std::signal(SIGBUS, on_segv);
  uint64_t *cpu_view = a.hostPointer ? (uint64_t *)a.hostPointer : dflag;
  *(volatile uint64_t *)cpu_view = 7;
  _mm_sfence();
  std::printf("CPU wrote device memory, reads back %llu\n",
              (unsigned long long)*(volatile uint64_t *)cpu_view);
  std::fflush(stdout);
  std::signal(SIGSEGV, SIG_DFL);
  std::signal(SIGBUS, SIG_DFL);
  run("flag in device memory (HBM poll)", cpu_view, dflag, reply, n);
  uint64_t *dkeys = nullptr;
  CHECK(hipExtMallocWithFlags((void **)&dkeys, 8192 * 8, hipDeviceMallocFinegrained));
  for (int K : {64, 256, 512, 1024}) {
    double best = 1e9;
    for (int r = 0; r < 50; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < K; ++i) ((volatile uint64_t *)dkeys)[i] = (uint64_t)(r * K + i);
      _mm_sfence();
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      best = us < best ? us : best;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < K; i += 2)
      _mm_stream_si128((__m128i *)(dkeys + i), _mm_set_epi64x((long long)i + 1, (long long)i));
    _mm_sfence();
    const double us2 = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    const auto t1 = std::chrono::steady_clock::now();
    const uint64_t back = ((volatile uint64_t *)dkeys)[K - 1];
    const double rb = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count();
    std::printf("CPU writes K=%5d keys into device memory: %7.2f us (best of 50, 8-byte stores), "
                "%7.2f us (16-byte streaming stores); one read back %6.2f us (%llu)\n",
                K, best, us2, rb, (unsigned long long)back);
  }
  keyreads("device memory", dkeys, reply + 4);
  CHECK(hipFree(dkeys));
  CHECK(hipFree(dflag));
  CHECK(hipHostFree(hflag));
  CHECK(hipHostFree(reply));
  return 0;
}
