// Probe of the rocprofiler-sdk device counting service on gfx950: which of
// the candidate counters exist, their dimensions (XCC / SE / ...), and
// whether consecutive samples are cumulative or per-interval.  Built and run
// by scripts/gpu_session.sh step "hwc"; output is informational only.
//
//   hipcc --offload-arch=gfx950 -O2 scripts/hwc_probe.hip -o /tmp/hwc_probe \
//         -I/opt/rocm/include -L/opt/rocm/lib -lrocprofiler-sdk
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace {
rocprofiler_context_id_t g_ctx{};
std::vector<rocprofiler_agent_id_t> g_gpus;
std::map<uint64_t, std::string> g_names;
std::vector<rocprofiler_counter_config_id_t> g_cfg;
const char* kWanted[] = {"SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE",
                         "GRBM_COUNT", "TCC_HIT", "TCC_MISS", "TCC_REQ", "TCC_EA0_RDREQ", "SQ_INSTS_LDS",
                         "SQ_INSTS_VMEM"};

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

rocprofiler_status_t on_counters(rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* ud) {
  auto* out = (std::vector<rocprofiler_counter_id_t>*)ud;
  for (size_t i = 0; i < n; ++i) {
    rocprofiler_counter_info_v1_t info{};
    info.size = sizeof(info);
    if (rocprofiler_query_counter_info(c[i], ROCPROFILER_COUNTER_INFO_VERSION_1, &info) != ROCPROFILER_STATUS_SUCCESS)
      continue;
    for (const char* w : kWanted)
      if (info.name && strcmp(info.name, w) == 0) {
        out->push_back(c[i]);
        g_names[c[i].handle] = info.name;
        printf("counter %-16s block=%s dims=", info.name, info.block ? info.block : "-");
        for (uint64_t d = 0; d < info.dimensions_count; ++d)
          printf("%s[%zu] ", info.dimensions[d]->name, info.dimensions[d]->instance_size);
        printf("\n");
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
  g_cfg.resize(g_gpus.size());
  for (size_t i = 0; i < g_gpus.size(); ++i) {
    std::vector<rocprofiler_counter_id_t> ids;
    CHK(rocprofiler_iterate_agent_supported_counters(g_gpus[i], on_counters, &ids));
    CHK(rocprofiler_create_counter_config(g_gpus[i], ids.data(), ids.size(), &g_cfg[i]));
    CHK(rocprofiler_configure_device_counting_service(g_ctx, rocprofiler_buffer_id_t{0}, g_gpus[i], set_cfg,
                                                      &g_cfg[i]));
  }
  return 0;
}

void tool_fini(void*) {}

rocprofiler_tool_configure_result_t* configure(uint32_t, const char*, uint32_t, rocprofiler_client_id_t* id) {
  id->name = "gpbs-hwc-probe";
  static rocprofiler_tool_configure_result_t r{sizeof(rocprofiler_tool_configure_result_t), tool_init, tool_fini,
                                               nullptr};
  return &r;
}

__global__ void busy(float* p, int iters) {
  float v = p[threadIdx.x];
  for (int i = 0; i < iters; ++i) v = v * 1.0001f + 0.5f;
  p[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

void sample(const char* tag) {
  std::vector<rocprofiler_counter_record_t> rec(8192);
  size_t n = rec.size();
  auto s = rocprofiler_sample_device_counting_service(g_ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE, rec.data(), &n);
  std::map<std::string, double> tot;
  std::map<std::string, size_t> cnt;
  for (size_t i = 0; i < n; ++i) {
    rocprofiler_counter_id_t cid{};
    rocprofiler_query_record_counter_id(rec[i].id, &cid);
    tot[g_names[cid.handle]] += rec[i].counter_value;
    cnt[g_names[cid.handle]]++;
  }
  printf("[%s] status=%d records=%zu\n", tag, (int)s, n);
  for (auto& kv : tot) printf("   %-16s sum=%.0f instances=%zu\n", kv.first.c_str(), kv.second, cnt[kv.first]);
}
}  // namespace

int main() {
  CHK(rocprofiler_force_configure(configure));
  hipSetDevice(0);
  float* d = nullptr;
  hipMalloc(&d, 1 << 24);
  hipMemset(d, 0, 1 << 24);
  CHK(rocprofiler_start_context(g_ctx));
  sample("start");
  sample("idle");
  hipLaunchKernelGGL(busy, dim3(4096), dim3(256), 0, 0, d, 20000);
  hipDeviceSynchronize();
  sample("after busy #1");
  hipLaunchKernelGGL(busy, dim3(4096), dim3(256), 0, 0, d, 20000);
  hipDeviceSynchronize();
  sample("after busy #2");
  sample("idle again");
  rocprofiler_stop_context(g_ctx);
  printf("done\n");
  return 0;
}
