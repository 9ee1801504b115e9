// N1 (health half): per-GPU health and telemetry through AMD SMI, with no HIP runtime.
//
// The reference's only node health signal was a container count over ssh (setup.sh:71-73)
// and the stuck-dashboard remediation (setup.sh:74-81). A GPU node needs more: the device
// plugin marks a device Unhealthy when its uncorrectable ECC count grows, and the node carries
// temperature / power / memory telemetry. AMD SMI reads sysfs and the DRM render node; it
// creates no KFD process, so the (GPU-clean) node agent can run it periodically — through the
// `tk8s-smi` tool, so a driver hiccup can never take the agent down with it.
#include "tk8s/smi.h"

#include <amd_smi/amdsmi.h>

#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "tk8s/json.h"

namespace tk8s {
namespace {

std::string status_str(amdsmi_status_t s) {
  const char* msg = nullptr;
  if (amdsmi_status_code_to_string(s, &msg) == AMDSMI_STATUS_SUCCESS && msg) return msg;
  return "amdsmi status " + std::to_string(static_cast<int>(s));
}

std::string bdf_str(const amdsmi_bdf_t& b) {
  char buf[32];
  std::snprintf(buf, sizeof buf, "%04llx:%02llx:%02llx.%llx",
                static_cast<unsigned long long>(b.domain_number), static_cast<unsigned long long>(b.bus_number),
                static_cast<unsigned long long>(b.device_number), static_cast<unsigned long long>(b.function_number));
  return buf;
}

const char* link_name(amdsmi_link_type_t t) {
  switch (t) {
    case AMDSMI_LINK_TYPE_XGMI: return "xgmi";
    case AMDSMI_LINK_TYPE_PCIE: return "pcie";
    case AMDSMI_LINK_TYPE_INTERNAL: return "internal";
    default: return "unknown";
  }
}

// Collects the metrics one GPU supports; a metric the platform does not expose is simply
// absent (listed under "unsupported") rather than an error.
std::string gpu_json(amdsmi_processor_handle h, int index) {
  Json j;
  std::vector<std::string> unsupported;
  j.kv("index", index);
  amdsmi_bdf_t bdf{};
  if (amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) j.kv("pci_bus_id", bdf_str(bdf));
  amdsmi_asic_info_t asic{};
  if (amdsmi_get_gpu_asic_info(h, &asic) == AMDSMI_STATUS_SUCCESS) {
    j.kv("market_name", std::string(asic.market_name));
    if (asic.num_of_compute_units != 0xFFFFFFFFu) j.kv("cu_count", asic.num_of_compute_units);
    if (asic.oam_id != 0xFFFFFFFFu) j.kv("oam_id", asic.oam_id);
    j.kv("asic_serial", std::string(asic.asic_serial));
  }
  amdsmi_driver_info_t drv{};
  if (amdsmi_get_gpu_driver_info(h, &drv) == AMDSMI_STATUS_SUCCESS)
    j.kv("driver", std::string(drv.driver_name) + " " + std::string(drv.driver_version));

  Json temps;
  bool any_temp = false;
  const std::pair<const char*, amdsmi_temperature_type_t> sensors[] = {
      {"edge", AMDSMI_TEMPERATURE_TYPE_EDGE},
      {"hotspot", AMDSMI_TEMPERATURE_TYPE_HOTSPOT},
      {"vram", AMDSMI_TEMPERATURE_TYPE_VRAM}};
  for (const auto& [name, type] : sensors) {
    int64_t c = 0;
    if (amdsmi_get_temp_metric(h, type, AMDSMI_TEMP_CURRENT, &c) == AMDSMI_STATUS_SUCCESS) {
      temps.kv(name, static_cast<int64_t>(c));
      any_temp = true;
    } else {
      unsupported.push_back(std::string("temp_") + name);
    }
  }
  if (any_temp) j.raw("temp_c", temps.str());

  amdsmi_power_info_t pw{};
  if (amdsmi_get_power_info(h, &pw) == AMDSMI_STATUS_SUCCESS) {
    Json p;
    // "not supported" shows up as all-ones of the field's width or of a 16-bit counter, and the
    // MI355X driver reports the limit in microwatts although the header says watts.
    auto valid = [](uint32_t v) { return v != 0xFFFFFFFFu && v != 0xFFFFu; };
    if (valid(pw.current_socket_power)) p.kv("current_w", pw.current_socket_power);
    if (valid(pw.average_socket_power)) p.kv("average_w", pw.average_socket_power);
    if (valid(pw.power_limit))
      p.kv("limit_w", pw.power_limit > 100000u ? pw.power_limit / 1000000u : pw.power_limit);
    j.raw("power", p.str());
  } else {
    unsupported.push_back("power");
  }

  uint64_t total = 0, used = 0;
  if (amdsmi_get_gpu_memory_total(h, AMDSMI_MEM_TYPE_VRAM, &total) == AMDSMI_STATUS_SUCCESS) {
    j.kv("vram_total_bytes", total);
    if (amdsmi_get_gpu_memory_usage(h, AMDSMI_MEM_TYPE_VRAM, &used) == AMDSMI_STATUS_SUCCESS)
      j.kv("vram_used_bytes", used);
  } else {
    unsupported.push_back("vram");
  }

  amdsmi_error_count_t ec{};
  const amdsmi_status_t es = amdsmi_get_gpu_total_ecc_count(h, &ec);
  if (es == AMDSMI_STATUS_SUCCESS) {
    j.raw("ecc", Json()
                     .kv("correctable", ec.correctable_count)
                     .kv("uncorrectable", ec.uncorrectable_count)
                     .kv("deferred", ec.deferred_count)
                     .str());
  } else {
    unsupported.push_back("ecc");
  }

  amdsmi_engine_usage_t act{};
  if (amdsmi_get_gpu_activity(h, &act) == AMDSMI_STATUS_SUCCESS) {
    Json a;
    if (act.gfx_activity != 0xFFFFFFFFu) a.kv("gfx_pct", act.gfx_activity);
    if (act.umc_activity != 0xFFFFFFFFu) a.kv("umc_pct", act.umc_activity);
    j.raw("activity", a.str());
  } else {
    unsupported.push_back("activity");
  }

  amdsmi_xgmi_info_t xg{};
  if (amdsmi_get_xgmi_info(h, &xg) == AMDSMI_STATUS_SUCCESS) {
    char hive[32];
    std::snprintf(hive, sizeof hive, "0x%llx", static_cast<unsigned long long>(xg.xgmi_hive_id));
    j.raw("xgmi", Json().kv("hive_id", std::string(hive)).kv("lanes", static_cast<int>(xg.xgmi_lanes)).str());
  } else {
    unsupported.push_back("xgmi");
  }

  // Healthy unless the hardware reports uncorrectable (or deferred) memory errors. Whether a
  // count is *new* is the agent's call: it compares against the count it saw at start-up.
  const bool healthy = es != AMDSMI_STATUS_SUCCESS || (ec.uncorrectable_count == 0 && ec.deferred_count == 0);
  j.kv("healthy", healthy);
  std::vector<std::string> quoted;
  for (const auto& u : unsupported) quoted.push_back("\"" + u + "\"");
  j.raw("unsupported", Json::array(quoted));
  return j.str();
}

}  // namespace

std::string smi_health_json(bool with_links) {
  const auto t0 = std::chrono::steady_clock::now();
  auto ms = [&] {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  const amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    return Json().kv("ok", false).kv("gpu_count", 0).kv("error", "amdsmi_init: " + status_str(st)).str();
  }
  std::vector<amdsmi_processor_handle> gpus;
  uint32_t nsock = 0;
  if (amdsmi_get_socket_handles(&nsock, nullptr) == AMDSMI_STATUS_SUCCESS && nsock > 0) {
    std::vector<amdsmi_socket_handle> socks(nsock);
    if (amdsmi_get_socket_handles(&nsock, socks.data()) == AMDSMI_STATUS_SUCCESS) {
      for (uint32_t s = 0; s < nsock; ++s) {
        uint32_t np = 0;
        if (amdsmi_get_processor_handles(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
        std::vector<amdsmi_processor_handle> ps(np);
        if (amdsmi_get_processor_handles(socks[s], &np, ps.data()) != AMDSMI_STATUS_SUCCESS) continue;
        for (uint32_t k = 0; k < np; ++k) {
          processor_type_t type{};
          if (amdsmi_get_processor_type(ps[k], &type) == AMDSMI_STATUS_SUCCESS &&
              type == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
            gpus.push_back(ps[k]);
        }
      }
    }
  }
  std::vector<std::string> devs;
  bool all_healthy = true;
  for (size_t i = 0; i < gpus.size(); ++i) {
    devs.push_back(gpu_json(gpus[i], static_cast<int>(i)));
    all_healthy = all_healthy && devs.back().find("\"healthy\":false") == std::string::npos;
  }
  std::vector<std::string> rows;
  if (with_links) {
    for (size_t i = 0; i < gpus.size(); ++i) {
      std::vector<std::string> row;
      for (size_t k = 0; k < gpus.size(); ++k) {
        if (i == k) {
          row.push_back(Json().kv("type", "self").kv("hops", 0).str());
          continue;
        }
        uint64_t hops = 0;
        amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
        const bool ok = amdsmi_topo_get_link_type(gpus[i], gpus[k], &hops, &t) == AMDSMI_STATUS_SUCCESS;
        row.push_back(Json().kv("type", ok ? link_name(t) : "unknown").kv("hops", static_cast<uint64_t>(ok ? hops : 0)).str());
      }
      rows.push_back(Json::array(row));
    }
  }
  amdsmi_version_t ver{};
  std::string lib;
  if (amdsmi_get_lib_version(&ver) == AMDSMI_STATUS_SUCCESS)
    lib = std::to_string(ver.major) + "." + std::to_string(ver.minor) + "." + std::to_string(ver.release);
  amdsmi_shut_down();
  Json out;
  out.kv("ok", !gpus.empty())
      .kv("healthy", all_healthy)
      .kv("gpu_count", static_cast<int>(gpus.size()))
      .kv("amdsmi_version", lib)
      .raw("gpus", Json::array(devs));
  if (with_links) out.raw("links", Json::array(rows));
  if (gpus.empty()) out.kv("error", "AMD SMI found no GPU");
  out.kv("ms", ms());
  return out.str();
}

}  // namespace tk8s
