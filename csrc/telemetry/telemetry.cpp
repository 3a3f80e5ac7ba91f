// GPU telemetry poller (N8): a background thread polls amd-smi for every
// MI355X on the node (HBM used/total, GFX and UMC busy %, uncorrectable ECC
// count) every `period_ms` and publishes a snapshot the load balancer and
// resource scheduler read without touching amd-smi themselves (amd-smi calls
// take ~ms; the router must never block on them).
//
// Reference equivalents: `Endpoint.Connections/ResponseTime/ErrorRate`
// (internal/loadbalancer/load_balancer.go:35-49) and `Resource.Load/Used`
// (internal/scheduler/resource_scheduler.go:35-47), which the reference never
// measures.  libamd_smi is dlopen'ed so the module builds and imports on
// hosts without a GPU (available() == false).  `inject()` overrides a field
// for fault-injection tests (slow GPU, HBM full, ECC storm, GPU lost).

#include <dlfcn.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "amd_smi/amdsmi.h"

namespace py = pybind11;

namespace {

struct GpuSample {
  bool valid = false;
  uint64_t hbm_total_mb = 0, hbm_used_mb = 0;
  uint32_t gfx_pct = 0, umc_pct = 0;
  uint64_t ecc_uncorrectable = 0;
  int64_t ts_ns = 0;
};

using init_t = amdsmi_status_t (*)(uint64_t);
using shut_t = amdsmi_status_t (*)(void);
using sockets_t = amdsmi_status_t (*)(uint32_t*, amdsmi_socket_handle*);
using procs_t = amdsmi_status_t (*)(amdsmi_socket_handle, uint32_t*, amdsmi_processor_handle*);
using vram_t = amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_vram_usage_t*);
using act_t = amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_engine_usage_t*);
using ecc_t = amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_gpu_block_t, amdsmi_error_count_t*);
using bdf_t = amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_bdf_t*);

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

class Telemetry {
 public:
  explicit Telemetry(int period_ms) : period_ms_(period_ms > 0 ? period_ms : 20) {
    const char* cands[] = {"libamd_smi.so", "/opt/rocm/lib/libamd_smi.so", "libamd_smi.so.26"};
    for (const char* c : cands) {
      lib_ = dlopen(c, RTLD_NOW | RTLD_LOCAL);
      if (lib_) break;
    }
    if (!lib_) {
      error_ = "libamd_smi not found";
      return;
    }
    init_ = (init_t)dlsym(lib_, "amdsmi_init");
    shut_ = (shut_t)dlsym(lib_, "amdsmi_shut_down");
    sockets_ = (sockets_t)dlsym(lib_, "amdsmi_get_socket_handles");
    procs_ = (procs_t)dlsym(lib_, "amdsmi_get_processor_handles");
    vram_ = (vram_t)dlsym(lib_, "amdsmi_get_gpu_vram_usage");
    act_ = (act_t)dlsym(lib_, "amdsmi_get_gpu_activity");
    ecc_ = (ecc_t)dlsym(lib_, "amdsmi_get_gpu_ecc_count");
    bdf_ = (bdf_t)dlsym(lib_, "amdsmi_get_gpu_device_bdf");
    if (!init_ || !sockets_ || !procs_ || !vram_) {
      error_ = "amd-smi symbols missing";
      return;
    }
    if (init_(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) {
      error_ = "amdsmi_init failed (no GPU?)";
      return;
    }
    inited_ = true;
    uint32_t ns = 0;
    if (sockets_(&ns, nullptr) != AMDSMI_STATUS_SUCCESS || ns == 0) {
      error_ = "no amd-smi sockets";
      return;
    }
    std::vector<amdsmi_socket_handle> socks(ns);
    sockets_(&ns, socks.data());
    for (auto s : socks) {
      uint32_t np = 0;
      if (procs_(s, &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
      std::vector<amdsmi_processor_handle> ps(np);
      procs_(s, &np, ps.data());
      for (auto p : ps) gpus_.push_back(p);
    }
    samples_.resize(gpus_.size());
    // PCI address of each amd-smi processor: the caller maps them to HIP
    // device indices (amd-smi enumerates every GPU of the node, HIP only the
    // visible ones, in possibly different order)
    for (auto p : gpus_) {
      int64_t key = -1;
      amdsmi_bdf_t b{};
      if (bdf_ && bdf_(p, &b) == AMDSMI_STATUS_SUCCESS)
        key = ((int64_t)b.domain_number << 16) | ((int64_t)b.bus_number << 8) | ((int64_t)b.device_number << 3) |
              (int64_t)b.function_number;
      bdfs_.push_back(key);
    }
    if (gpus_.empty()) error_ = "no GPUs found";
  }

  ~Telemetry() {
    stop();
    if (inited_ && shut_) shut_();
    // libamd_smi stays loaded: unloading it under live threads is unsafe
  }

  bool available() const { return !gpus_.empty(); }
  std::string error() const { return error_; }
  int count() const { return (int)gpus_.size(); }

  void poll_once() {
    for (size_t i = 0; i < gpus_.size(); ++i) {
      GpuSample s;
      amdsmi_vram_usage_t v{};
      if (vram_(gpus_[i], &v) == AMDSMI_STATUS_SUCCESS) {
        s.valid = true;
        s.hbm_total_mb = v.vram_total;
        s.hbm_used_mb = v.vram_used;
      }
      if (act_) {
        amdsmi_engine_usage_t a{};
        if (act_(gpus_[i], &a) == AMDSMI_STATUS_SUCCESS) {
          s.gfx_pct = a.gfx_activity;
          s.umc_pct = a.umc_activity;
        }
      }
      if (ecc_) {
        amdsmi_error_count_t e{};
        if (ecc_(gpus_[i], AMDSMI_GPU_BLOCK_UMC, &e) == AMDSMI_STATUS_SUCCESS) s.ecc_uncorrectable = e.uncorrectable_count;
      }
      s.ts_ns = now_ns();
      std::lock_guard<std::mutex> lk(mu_);
      samples_[i] = s;
    }
    polls_++;
  }

  void start() {
    if (th_.joinable() || !available()) return;
    stop_ = false;
    th_ = std::thread([this] {
      while (!stop_.load()) {
        poll_once();
        std::this_thread::sleep_for(std::chrono::milliseconds(period_ms_));
      }
    });
  }

  void stop() {
    stop_ = true;
    if (th_.joinable()) {
      py::gil_scoped_release nogil;
      th_.join();
    }
  }

  void inject(int gpu, const std::string& field, double value) {
    std::lock_guard<std::mutex> lk(mu_);
    overrides_[{gpu, field}] = value;
  }
  void clear_injections() {
    std::lock_guard<std::mutex> lk(mu_);
    overrides_.clear();
  }

  py::list snapshot(int synthetic) {
    std::vector<GpuSample> cp;
    std::map<std::pair<int, std::string>, double> ov;
    {
      std::lock_guard<std::mutex> lk(mu_);
      cp = samples_;
      ov = overrides_;
    }
    if (cp.empty() && synthetic > 0) cp.resize(synthetic);  // no GPU: fault-injection playground
    py::list out;
    for (size_t i = 0; i < cp.size(); ++i) {
      py::dict d;
      d["gpu"] = (int)i;
      d["valid"] = cp[i].valid;
      d["hbm_total_mb"] = cp[i].hbm_total_mb;
      d["hbm_used_mb"] = cp[i].hbm_used_mb;
      d["gfx_pct"] = cp[i].gfx_pct;
      d["umc_pct"] = cp[i].umc_pct;
      d["ecc_uncorrectable"] = cp[i].ecc_uncorrectable;
      d["ts_ns"] = cp[i].ts_ns;
      d["pci"] = i < bdfs_.size() ? bdfs_[i] : (int64_t)-1;
      for (auto& kv : ov) {
        if (kv.first.first != (int)i) continue;
        if (kv.first.second == "valid") d["valid"] = kv.second != 0.0;
        else d[kv.first.second.c_str()] = (int64_t)kv.second;
      }
      out.append(d);
    }
    return out;
  }

  int64_t polls() const { return polls_.load(); }
  std::vector<int64_t> pci_addresses() const { return bdfs_; }

 private:
  void* lib_ = nullptr;
  bool inited_ = false;
  std::string error_;
  init_t init_ = nullptr;
  shut_t shut_ = nullptr;
  sockets_t sockets_ = nullptr;
  procs_t procs_ = nullptr;
  vram_t vram_ = nullptr;
  act_t act_ = nullptr;
  ecc_t ecc_ = nullptr;
  bdf_t bdf_ = nullptr;
  std::vector<int64_t> bdfs_;    // domain<<16 | bus<<8 | device<<3 | function
  std::vector<amdsmi_processor_handle> gpus_;
  std::vector<GpuSample> samples_;
  std::map<std::pair<int, std::string>, double> overrides_;
  std::mutex mu_;
  std::thread th_;
  std::atomic<bool> stop_{false};
  std::atomic<int64_t> polls_{0};
  int period_ms_;
};

}  // namespace

PYBIND11_MODULE(_telemetry, m) {
  m.doc() = "amd-smi telemetry poller (N8)";
  py::class_<Telemetry>(m, "Telemetry")
      .def(py::init<int>(), py::arg("period_ms") = 20)
      .def("available", &Telemetry::available)
      .def("error", &Telemetry::error)
      .def("count", &Telemetry::count)
      .def("poll_once", &Telemetry::poll_once, py::call_guard<py::gil_scoped_release>())
      .def("start", &Telemetry::start)
      .def("stop", &Telemetry::stop)
      .def("inject", &Telemetry::inject)
      .def("clear_injections", &Telemetry::clear_injections)
      .def("snapshot", &Telemetry::snapshot, py::arg("synthetic") = 0)
      .def("polls", &Telemetry::polls)
      .def("pci_addresses", [](Telemetry& t) { return t.pci_addresses(); });
}
