// N1 health: AMD SMI telemetry per GPU (no HIP runtime, no KFD process).
#pragma once

#include <string>

namespace tk8s {

// {"ok":..,"healthy":..,"gpu_count":n,"gpus":[{"pci_bus_id","temp_c","power","vram_*","ecc",
// "activity","xgmi","healthy","unsupported"}..],"links":[[{"type","hops"}..]..],"ms":..}.
// Never throws; a host without GPUs (or without the amdgpu driver) yields ok=false + "error".
std::string smi_health_json(bool with_links = true);

}  // namespace tk8s
