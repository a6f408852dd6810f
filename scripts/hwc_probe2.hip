// Probe #2 of the rocprofiler-sdk device counting service on gfx950: can the
// per-tenant vPMU be built from OWNERSHIP instead of a model?
//
//  1. `list`: every hardware (non-derived) SQ/TCP/TCC/GRBM/TA counter and its
//     dimensions (which counters resolve per shader engine / per CU).
//  2. `sep`: a VALU-bound kernel confined (CU mask) to shader engines {0,1} of
//     every XCD and an HBM-stream kernel confined to SEs {2,3}, alone and
//     together; counter deltas are printed per (XCC, SE) so it is visible
//     whether SE-resolved counters separate the two tenants exactly.
//  3. `lat`: synchronous sample latency (median / p99 / max over 200 samples)
//     and the stream kernel's bandwidth with and without a 1 kHz sampler.
//
//   hipcc --offload-arch=gfx950 -O2 scripts/hwc_probe2.hip -o scripts/hwc_probe2.bin \
//         -I/opt/rocm/include -L/opt/rocm/lib -lrocprofiler-sdk
//   scripts/hwc_probe2.bin list|sep|lat  [counter,counter,...]
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

namespace {
rocprofiler_context_id_t g_ctx{};
std::vector<rocprofiler_agent_id_t> g_gpus;
std::map<uint64_t, std::string> g_names;
std::vector<rocprofiler_counter_config_id_t> g_cfg;
std::vector<std::string> g_want;
std::string g_mode = "sep";
rocprofiler_counter_dimension_id_t g_dim_xcc{}, g_dim_se{}, g_dim_inst{};
bool g_have_xcc = false, g_have_se = false, g_have_inst = false;

#define CHK(x)                                                                            \
  do {                                                                                    \
    auto _s = (x);                                                                        \
    if (_s != ROCPROFILER_STATUS_SUCCESS) fprintf(stderr, "%s -> %d\n", #x, (int)_s); \
  } while (0)

rocprofiler_status_t on_agents(rocprofiler_agent_version_t, const void** agents, size_t n, void*) {
  for (size_t i = 0; i < n; ++i) {
    auto* a = (const rocprofiler_agent_v0_t*)agents[i];
    if (a->type == ROCPROFILER_AGENT_TYPE_GPU) g_gpus.push_back(a->id);
  }
  return ROCPROFILER_STATUS_SUCCESS;
}

bool listed_block(const char* n) {
  for (const char* p : {"SQ_", "TCP_", "TCC_", "GRBM_", "TA_", "TD_", "CPC_", "SPI_"})
    if (std::strncmp(n, p, std::strlen(p)) == 0) return true;
  return false;
}

rocprofiler_status_t on_counters(rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* ud) {
  auto* out = (std::vector<rocprofiler_counter_id_t>*)ud;
  for (size_t i = 0; i < n; ++i) {
    rocprofiler_counter_info_v1_t info{};
    info.size = sizeof(info);
    if (rocprofiler_query_counter_info(c[i], ROCPROFILER_COUNTER_INFO_VERSION_1, &info) != ROCPROFILER_STATUS_SUCCESS ||
        !info.name)
      continue;
    if (g_mode == "list" && listed_block(info.name)) {
      printf("counter %-32s derived=%d block=%-6s dims=", info.name, (int)info.is_derived,
             info.block ? info.block : "-");
      for (uint64_t d = 0; d < info.dimensions_count; ++d)
        printf("%s[%zu] ", info.dimensions[d]->name, info.dimensions[d]->instance_size);
      printf("\n");
    }
    for (auto& w : g_want)
      if (w == info.name) {
        out->push_back(c[i]);
        g_names[c[i].handle] = info.name;
        for (uint64_t d = 0; d < info.dimensions_count; ++d) {
          const char* dn = info.dimensions[d]->name;
          if (!std::strcmp(dn, "DIMENSION_XCC")) g_dim_xcc = info.dimensions[d]->id, g_have_xcc = true;
          if (!std::strcmp(dn, "DIMENSION_SHADER_ENGINE")) g_dim_se = info.dimensions[d]->id, g_have_se = true;
          if (!std::strcmp(dn, "DIMENSION_INSTANCE")) g_dim_inst = info.dimensions[d]->id, g_have_inst = true;
        }
      }
  }
  return ROCPROFILER_STATUS_SUCCESS;
}

void set_cfg(rocprofiler_context_id_t ctx, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t set,
             void* ud) {
  CHK(set(ctx, *(rocprofiler_counter_config_id_t*)ud));
}

int tool_init(rocprofiler_client_finalize_t, void*) {
  CHK(rocprofiler_create_context(&g_ctx));
  CHK(rocprofiler_query_available_agents(ROCPROFILER_AGENT_INFO_VERSION_0, on_agents, sizeof(rocprofiler_agent_v0_t),
                                         nullptr));
  if (g_gpus.empty()) return 0;
  g_gpus.resize(1);
  g_cfg.resize(1);
  std::vector<rocprofiler_counter_id_t> ids;
  CHK(rocprofiler_iterate_agent_supported_counters(g_gpus[0], on_counters, &ids));
  if (ids.empty()) return 0;
  CHK(rocprofiler_create_counter_config(g_gpus[0], ids.data(), ids.size(), &g_cfg[0]));
  CHK(rocprofiler_configure_device_counting_service(g_ctx, rocprofiler_buffer_id_t{0}, g_gpus[0], set_cfg, &g_cfg[0]));
  return 0;
}

void tool_fini(void*) {}

rocprofiler_tool_configure_result_t* configure(uint32_t, const char*, uint32_t, rocprofiler_client_id_t* id) {
  id->name = "gpbs-hwc-probe2";
  static rocprofiler_tool_configure_result_t r{sizeof(rocprofiler_tool_configure_result_t), tool_init, tool_fini,
                                               nullptr};
  return &r;
}

__global__ __launch_bounds__(256) void k_valu(float* p, int iters) {
  float a = p[threadIdx.x] + 1.f, b = a * 0.5f, c = a + 2.f, d = b - 1.f;
  for (int i = 0; i < iters; ++i) {
    a = a * 1.0001f + 0.5f;
    b = b * 0.9999f + a;
    c = c * 1.0002f - b;
    d = d * 0.9998f + c;
  }
  if (a + b + c + d == 1234.5f) p[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

typedef float f4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream(const f4* __restrict__ s, f4* __restrict__ d, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

hipStream_t se_stream(unsigned se_bits) {
  uint32_t m[8] = {};
  for (int b = 0; b < 256; ++b)
    if (se_bits & (1u << ((b / 8) % 4))) m[b / 32] |= 1u << (b % 32);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, 8, m) != hipSuccess) {
    fprintf(stderr, "cumask stream failed\n");
    exit(1);
  }
  return s;
}

using Key = std::tuple<std::string, int, int>;  // counter, xcc, se
std::map<Key, double> sample_map(double* us = nullptr) {
  static std::vector<rocprofiler_counter_record_t> rec(1 << 16);
  size_t n = rec.size();
  auto t0 = std::chrono::steady_clock::now();
  auto s = rocprofiler_sample_device_counting_service(g_ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE, rec.data(), &n);
  if (us) *us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  std::map<Key, double> m;
  if (s != ROCPROFILER_STATUS_SUCCESS) {
    fprintf(stderr, "sample -> %d\n", (int)s);
    return m;
  }
  for (size_t i = 0; i < n; ++i) {
    rocprofiler_counter_id_t cid{};
    rocprofiler_query_record_counter_id(rec[i].id, &cid);
    size_t x = 0, se = 0;
    if (g_have_xcc) rocprofiler_query_record_dimension_position(rec[i].id, g_dim_xcc, &x);
    if (g_have_se && rocprofiler_query_record_dimension_position(rec[i].id, g_dim_se, &se) != ROCPROFILER_STATUS_SUCCESS)
      se = 99;
    m[Key(g_names[cid.handle], (int)x, (int)se)] += rec[i].counter_value;
  }
  return m;
}

void print_delta(const char* tag, const std::map<Key, double>& a, const std::map<Key, double>& b) {
  printf("== %s\n", tag);
  std::map<std::string, std::map<int, double>> by_se;  // counter -> se -> sum over xcc
  std::map<std::string, std::map<int, double>> by_x;
  for (auto& kv : b) {
    auto it = a.find(kv.first);
    const double d = kv.second - (it == a.end() ? 0 : it->second);
    by_se[std::get<0>(kv.first)][std::get<2>(kv.first)] += d;
    by_x[std::get<0>(kv.first)][std::get<1>(kv.first)] += d;
  }
  for (auto& c : by_se) {
    printf("  %-28s by_se:", c.first.c_str());
    for (auto& s : c.second) printf(" se%d=%.4g", s.first, s.second);
    printf("   by_xcc:");
    for (auto& x : by_x[c.first]) printf(" %.3g", x.second);
    printf("\n");
  }
  fflush(stdout);
}

void run_for(double ms, hipStream_t sv, hipStream_t ss, float* p, const f4* src, f4* dst, size_t n4) {
  auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() < ms) {
    if (sv) hipLaunchKernelGGL(k_valu, dim3(2048), dim3(256), 0, sv, p, 4000);
    if (ss) hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, ss, src, dst, n4);
    if (sv) hipStreamSynchronize(sv);
    if (ss) hipStreamSynchronize(ss);
  }
}
}  // namespace

int main(int argc, char** argv) {
  g_mode = argc > 1 ? argv[1] : "sep";
  std::string list = argc > 2 ? argv[2]
                              : "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_BUSY_CYCLES,"
                                "SQ_WAVE_CYCLES,SQ_INSTS_LDS,SQ_WAVES,TCC_REQ,TCC_MISS,TCP_TCC_READ_REQ,"
                                "TCP_TCC_WRITE_REQ,GRBM_GUI_ACTIVE";
  for (size_t p = 0; p < list.size();) {
    size_t e = list.find(',', p);
    g_want.push_back(list.substr(p, e == std::string::npos ? std::string::npos : e - p));
    p = e == std::string::npos ? list.size() : e + 1;
  }
  CHK(rocprofiler_force_configure(configure));
  hipSetDevice(0);
  if (g_mode == "list") {
    printf("list done\n");
    return 0;
  }
  printf("dims: xcc=%d se=%d inst=%d\n", g_have_xcc, g_have_se, g_have_inst);
  const size_t bytes = 512ull << 20, n4 = bytes / 16;
  float *p = nullptr, *src = nullptr, *dst = nullptr;
  hipMalloc(&p, 2048 * 256 * 4);
  hipMalloc(&src, bytes);
  hipMalloc(&dst, bytes);
  hipMemset(p, 0, 2048 * 256 * 4);
  hipMemset(src, 0, bytes);
  hipStream_t s01 = se_stream(0x3), s23 = se_stream(0xC);
  CHK(rocprofiler_start_context(g_ctx));
  if (g_mode == "sep") {
    auto m0 = sample_map();
    run_for(30, s01, nullptr, p, (f4*)src, (f4*)dst, n4);
    auto m1 = sample_map();
    print_delta("valu on SE{0,1} alone", m0, m1);
    run_for(30, nullptr, s23, p, (f4*)src, (f4*)dst, n4);
    auto m2 = sample_map();
    print_delta("stream on SE{2,3} alone", m1, m2);
    run_for(30, s01, s23, p, (f4*)src, (f4*)dst, n4);
    auto m3 = sample_map();
    print_delta("valu SE{0,1} + stream SE{2,3}", m2, m3);
    hipDeviceSynchronize();
    auto m4 = sample_map();
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    auto m5 = sample_map();
    print_delta("idle 20 ms", m4, m5);
  } else if (g_mode == "lat") {
    std::vector<double> us;
    for (int i = 0; i < 200; ++i) {
      double u = 0;
      sample_map(&u);
      us.push_back(u);
    }
    std::sort(us.begin(), us.end());
    printf("sync sample latency idle: p50 %.1f us  p99 %.1f us  max %.1f us\n", us[100], us[198], us[199]);
    // bandwidth with / without a 1 kHz sampler
    hipStream_t sf = nullptr;
    hipStreamCreateWithFlags(&sf, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int mode = 0; mode < 3; ++mode) {
      std::atomic<bool> stop{false};
      std::vector<double> lus;
      std::thread th;
      if (mode > 0)
        th = std::thread([&] {
          while (!stop) {
            double u = 0;
            sample_map(&u);
            lus.push_back(u);
            if (mode == 1) std::this_thread::sleep_for(std::chrono::microseconds(1000));
          }
        });
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, sf, (f4*)src, (f4*)dst, n4);
      hipEventRecord(e0, sf);
      for (int it = 0; it < 100; ++it)
        hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, sf, (f4*)src, (f4*)dst, n4);
      hipEventRecord(e1, sf);
      hipEventSynchronize(e1);
      stop = true;
      if (th.joinable()) th.join();
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      std::sort(lus.begin(), lus.end());
      printf("stream copy %s: %.3f TB/s (rd+wr)  samples=%zu p50=%.1f us max=%.1f us\n",
             mode == 0 ? "no sampler" : mode == 1 ? "1 kHz sampler" : "back-to-back sampler",
             2.0 * bytes * 100 / (ms * 1e-3) / 1e12, lus.size(), lus.empty() ? 0 : lus[lus.size() / 2],
             lus.empty() ? 0 : lus.back());
    }
  }
  rocprofiler_stop_context(g_ctx);
  printf("done\n");
  return 0;
}
