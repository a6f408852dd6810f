// Probe: can the host write the partition table straight into device memory
// (large-BAR mapping of an uncached / fine-grained VRAM allocation), so a
// switch needs no kernel and no queue?  Each method runs in a forked child
// (the parent never touches the GPU): allocate, obtain a host pointer, store
// from the host, and read it back on the device with a polling kernel.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/bar_probe.hip -o /tmp/bar_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/wait.h>
#include <unistd.h>
#include <x86intrin.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

__global__ void k_poll(const unsigned* p, unsigned want, unsigned* out, unsigned long long max_iter) {
  unsigned v = 0;
  unsigned long long i = 0;
  for (; i < max_iter; ++i) {
    v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == want) break;
    __builtin_amdgcn_s_sleep(1);
  }
  out[0] = v;
  out[1] = (unsigned)i;
}

static int check_device_sees(unsigned* dptr, volatile unsigned* hptr) {
  unsigned* out = nullptr;
  if (hipHostMalloc((void**)&out, 8, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return -1;
  out[0] = out[1] = 0xdead;
  hptr[0] = 0;
  _mm_sfence();
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipLaunchKernelGGL(k_poll, dim3(1), dim3(64), 0, s, (const unsigned*)dptr, 0x1234u, out, 200000000ull);
  std::this_thread::sleep_for(std::chrono::milliseconds(50));  // kernel polling
  const auto t0 = std::chrono::steady_clock::now();
  hptr[0] = 0x1234u;
  _mm_sfence();
  while (__atomic_load_n(&out[0], __ATOMIC_ACQUIRE) == 0xdead &&
         std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5)) {
  }
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  hipStreamSynchronize(s);
  printf("    device saw 0x%x after %u polls, host observed ack after %.1f us\n", out[0], out[1], us);
  const int ok = out[0] == 0x1234u;
  hipStreamDestroy(s);
  hipHostFree(out);
  return ok ? 0 : 1;
}

static int method_hip(unsigned flags, const char* name) {
  unsigned* d = nullptr;
  if (hipExtMallocWithFlags((void**)&d, 4096, flags) != hipSuccess) {
    printf("  %s: alloc failed\n", name);
    return 2;
  }
  hipPointerAttribute_t a;
  std::memset(&a, 0, sizeof(a));
  hipPointerGetAttributes(&a, d);
  printf("  %s: dev %p hostPointer %p\n", name, (void*)d, a.hostPointer);
  if (!a.hostPointer) return 3;
  return check_device_sees(d, (volatile unsigned*)a.hostPointer);
}

struct Pools {
  hsa_agent_t gpu{}, cpu{};
  hsa_amd_memory_pool_t fine{};
  bool have_gpu = false, have_cpu = false, have_fine = false;
};

static hsa_status_t pool_cb(hsa_amd_memory_pool_t p, void* ud) {
  auto* P = (Pools*)ud;
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t fl = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !P->have_fine) {
    P->fine = p;
    P->have_fine = true;
  }
  return HSA_STATUS_SUCCESS;
}

static hsa_status_t agent_cb(hsa_agent_t a, void* ud) {
  auto* P = (Pools*)ud;
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !P->have_gpu) {
    P->gpu = a;
    P->have_gpu = true;
    hsa_amd_agent_iterate_memory_pools(a, pool_cb, P);
  }
  if (t == HSA_DEVICE_TYPE_CPU && !P->have_cpu) {
    P->cpu = a;
    P->have_cpu = true;
  }
  return HSA_STATUS_SUCCESS;
}

static int method_hsa() {
  hipFree(nullptr);  // runtime up (initialises HSA)
  Pools P;
  hsa_iterate_agents(agent_cb, &P);
  printf("  hsa: gpu %d cpu %d fine-grained VRAM pool %d\n", P.have_gpu, P.have_cpu, P.have_fine);
  if (!P.have_fine) return 3;
  void* d = nullptr;
  if (hsa_amd_memory_pool_allocate(P.fine, 4096, 0, &d) != HSA_STATUS_SUCCESS) return 2;
  hsa_agent_t both[2] = {P.gpu, P.cpu};
  const hsa_status_t st = hsa_amd_agents_allow_access(2, both, nullptr, d);
  printf("  hsa: ptr %p allow_access(cpu,gpu) status %d\n", d, (int)st);
  if (st != HSA_STATUS_SUCCESS) return 4;
  return check_device_sees((unsigned*)d, (volatile unsigned*)d);
}

int main() {
  const char* names[] = {"hipDeviceMallocUncached", "hipDeviceMallocFinegrained", "hsa fine-grained VRAM pool"};
  for (int m = 0; m < 3; ++m) {
    printf("method %s\n", names[m]);
    fflush(stdout);
    const pid_t pid = fork();
    if (pid == 0) {
      alarm(30);
      int rc = m == 0 ? method_hip(hipDeviceMallocUncached, names[m])
               : m == 1 ? method_hip(hipDeviceMallocFinegrained, names[m])
                        : method_hsa();
      fflush(stdout);
      _exit(rc);
    }
    int st = 0;
    waitpid(pid, &st, 0);
    printf("  -> %s\n", WIFEXITED(st) ? (WEXITSTATUS(st) == 0 ? "OK" : "failed") : "child killed by signal");
    fflush(stdout);
  }
  return 0;
}
