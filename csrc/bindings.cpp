// pybind11 bindings: `otedama_amd._native`.
//
// Exposes the host SHA-256 / scrypt primitives, the per-job folding for the
// gfx950 kernels, raw kernel launches (for torch-owned buffers / streams), and
// the native GpuMiner / CpuMiner runtime objects.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <array>
#include <atomic>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "otedama/aead.h"
#include "otedama/job.h"
#include "otedama/runtime.h"
#include "otedama/trace.h"
#include "otedama/sha256.h"
#include "otedama/sv2_frame.h"
#include "otedama/clock_bounds.h"
#include "otedama/work_queue.h"
#include "otedama/x11.h"

namespace py = pybind11;
using namespace otedama;

namespace otedama {
void py_launch_sha256d(const Sha256dParams& p, uint32_t base, uint64_t count, uintptr_t out, uint32_t cap, int grid,
                       uintptr_t stream);
void py_launch_sha256d_k(const Sha256dParamsK& p, uint32_t base, uint64_t count, uintptr_t out, uint32_t cap, int grid,
                         uintptr_t stream);
void py_launch_sha256d_v(const Sha256dParamsV& p, uintptr_t vars, uint32_t base, uint64_t count, uintptr_t out,
                         uint32_t cap, int grid, uintptr_t stream, int block, int chains);
void py_launch_scrypt(const ScryptParams& p, uint32_t base, uint32_t count, uintptr_t xbuf, uintptr_t scratch, int gap,
                      uintptr_t out, uint32_t cap, int grid, uintptr_t stream);
void py_launch_x11_stage(const X11Params& p, int stage, uint32_t base, uintptr_t H, uint32_t stride, uint32_t n,
                         uintptr_t out, uint32_t cap, uintptr_t stream);
void py_launch_x11(const X11Params& p, uint32_t base, uintptr_t H, uint32_t stride, uint32_t n, uintptr_t out,
                   uint32_t cap, uintptr_t stream);
uint64_t scrypt_scratch_bytes(int grid, int gap);
int gpu_device_count();
std::string gpu_arch_name(int device);
int gpu_cu_count(int device);
}  // namespace otedama

namespace {

std::string need(const py::bytes& b, size_t n, const char* what) {
  std::string s = b;
  if (s.size() != n) throw std::invalid_argument(std::string(what) + ": expected " + std::to_string(n) + " bytes");
  return s;
}

py::bytes to_bytes(const uint8_t* p, size_t n) { return py::bytes(reinterpret_cast<const char*>(p), n); }

std::shared_ptr<JobTemplate> make_job(const py::dict& d) {
  auto j = std::make_shared<JobTemplate>();
  auto get = [&](const char* k) -> py::object {
    if (d.contains(k)) return py::object(d[k]);
    return py::none();
  };
  std::string hdr = need(d["header"].cast<py::bytes>(), 80, "header");
  std::memcpy(j->header, hdr.data(), 80);
  std::string tgt = need(d["target"].cast<py::bytes>(), 32, "target");
  std::memcpy(j->target, tgt.data(), 32);
  if (!get("epoch").is_none()) j->epoch = d["epoch"].cast<uint64_t>();
  if (!get("job_id").is_none()) j->job_id = d["job_id"].cast<std::string>();
  if (!get("channel_id").is_none()) j->channel_id = d["channel_id"].cast<uint32_t>();
  if (!get("algo").is_none()) {
    auto a = d["algo"].cast<std::string>();
    if (a == "sha256d") j->algo = Algo::kSha256d;
    else if (a == "scrypt") j->algo = Algo::kScrypt;
    else if (a == "x11") j->algo = Algo::kX11;
    else throw std::invalid_argument("unsupported algo for the native miner: " + a);
  }
  if (!get("version_mask").is_none()) j->version_mask = d["version_mask"].cast<uint32_t>();
  if (!get("ntime_roll").is_none()) j->ntime_roll = d["ntime_roll"].cast<uint32_t>();
  if (!get("coinb1").is_none()) {
    j->has_coinbase = true;
    std::string c1 = d["coinb1"].cast<py::bytes>(), c2 = d["coinb2"].cast<py::bytes>();
    std::string e1 = d["extranonce1"].cast<py::bytes>();
    j->coinb1.assign(c1.begin(), c1.end());
    j->coinb2.assign(c2.begin(), c2.end());
    j->extranonce1.assign(e1.begin(), e1.end());
    j->extranonce2_size = d["extranonce2_size"].cast<uint32_t>();
    for (auto& br : d["merkle_branches"].cast<py::list>()) {
      std::string b = br.cast<py::bytes>();
      j->merkle_branches.emplace_back(b.begin(), b.end());
    }
  }
  if (!get("variant_start").is_none()) j->variant_start = d["variant_start"].cast<uint64_t>();
  if (!get("variant_stride").is_none()) j->variant_stride = d["variant_stride"].cast<uint64_t>();
  if (j->variant_stride == 0) j->variant_stride = 1;
  return j;
}

py::list shares_to_list(std::vector<ShareRecord>&& v) {
  py::list out;
  for (auto& s : v) {
    py::dict d;
    d["epoch"] = s.epoch;
    d["job_id"] = s.job_id;
    d["channel_id"] = s.channel_id;
    d["nonce"] = s.nonce;
    d["ntime"] = s.ntime;
    d["version"] = s.version;
    d["extranonce2"] = s.extranonce2;
    d["extranonce2_size"] = s.extranonce2_size;
    d["hash"] = to_bytes(s.hash, 32);
    d["device_id"] = s.device_id;
    d["found_at"] = s.found_at;
    d["device_found_at"] = s.device_found_at;
    out.append(d);
  }
  return out;
}

py::dict stats_to_dict(const MinerStats& s) {
  py::dict d;
  d["hashes"] = s.hashes;
  d["candidates"] = s.candidates;
  d["shares"] = s.shares;
  d["dropped"] = s.dropped;
  d["launches"] = s.launches;
  d["rejected_candidates"] = s.rejected_candidates;
  d["variant_launches"] = s.variant_launches;
  d["busy_seconds"] = s.busy_seconds;
  d["faulted"] = s.faulted;
  d["error"] = s.error;
  d["variant_next"] = s.variant_next;
  d["variant_epoch"] = s.variant_epoch;
  d["job_switches"] = s.job_switches;
  d["last_job_switch_ms"] = s.last_job_switch_ms;
  d["job_switch_ms"] = s.job_switch_ms;
  d["work_started"] = s.work_started;
  d["reserved_cus"] = s.reserved_cus;
  d["ring_overflow"] = s.ring_overflow;
  d["verify_dropped"] = s.verify_dropped;
  d["verify_queue_peak"] = s.verify_queue_peak;
  d["launch_hashes"] = s.launch_hashes;
  d["aborted_launches"] = s.aborted_launches;
  d["ring_hits"] = s.ring_hits;
  d["clock_calib_rtt_us"] = s.clock_calib_rtt_us;
  d["clock_samples"] = s.clock_samples;
  d["host_abort"] = s.host_abort;
  d["hashes_done_at_s"] = s.hashes_done_at_s;
  {
    py::dict ph;
    for (const auto& kv : s.startup_ms) ph[py::str(kv.first)] = kv.second;
    d["startup_ms"] = ph;
    py::dict rs;
    for (const auto& kv : s.startup_rss_mb) rs[py::str(kv.first)] = kv.second;
    d["startup_rss_mb"] = rs;
  }
  return d;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "Otedama MI355X native runtime (gfx950 HIP kernels + C++ host runtime)";

  m.def("cpu_has_sha_ni", &cpu_has_sha_ni);
  m.def("sha256", [](const py::bytes& b) {
    std::string s = b; uint8_t o[32];
    sha256(reinterpret_cast<const uint8_t*>(s.data()), s.size(), o);
    return to_bytes(o, 32);
  });
  m.def("sha256d", [](const py::bytes& b) {
    std::string s = b; uint8_t o[32];
    { py::gil_scoped_release r; sha256d(reinterpret_cast<const uint8_t*>(s.data()), s.size(), o); }
    return to_bytes(o, 32);
  });
  m.def("hmac_sha256", [](const py::bytes& k, const py::bytes& msg) {
    std::string ks = k, ms = msg; uint8_t o[32];
    hmac_sha256(reinterpret_cast<const uint8_t*>(ks.data()), ks.size(),
                reinterpret_cast<const uint8_t*>(ms.data()), ms.size(), o);
    return to_bytes(o, 32);
  });
  m.def("aead_seal", [](int kind, const py::bytes& key, const py::bytes& nonce, const py::bytes& plain,
                        const py::bytes& aad) {
    std::string out = aead_seal(static_cast<AeadKind>(kind), key, nonce, plain, aad);
    return py::bytes(out);
  }, py::arg("kind"), py::arg("key"), py::arg("nonce"), py::arg("plain"), py::arg("aad") = py::bytes());
  m.def("aead_open", [](int kind, const py::bytes& key, const py::bytes& nonce, const py::bytes& sealed,
                        const py::bytes& aad) -> py::object {
    std::string out;
    if (!aead_open(static_cast<AeadKind>(kind), key, nonce, sealed, aad, &out)) return py::none();
    return py::bytes(out);
  }, py::arg("kind"), py::arg("key"), py::arg("nonce"), py::arg("sealed"), py::arg("aad") = py::bytes());
  m.attr("SCRYPT_COOP") = kScryptCoop;
  m.attr("SCRYPT_LANE_W8") = kScryptLaneW8;
  m.attr("SCRYPT_COOP2") = kScryptCoop2;
  m.attr("SCRYPT_COOP_SPLIT") = kScryptCoopSplit;
  m.attr("AEAD_AES256GCM") = 0;
  m.attr("AEAD_CHACHA20POLY1305") = 1;
  m.def("scrypt_1024_1_1_batch", [](const std::vector<py::bytes>& hs) {
    std::vector<std::string> in;
    for (const auto& h : hs) in.push_back(need(h, 80, "header"));
    std::vector<std::array<uint8_t, 32>> out(in.size());
    std::vector<const uint8_t*> ip;
    std::vector<uint8_t*> op;
    for (size_t i = 0; i < in.size(); ++i) {
      ip.push_back(reinterpret_cast<const uint8_t*>(in[i].data()));
      op.push_back(out[i].data());
    }
    {
      py::gil_scoped_release r;
      scrypt_1024_1_1_batch(int(in.size()), ip.data(), op.data());
    }
    py::list res;
    for (const auto& o : out) res.append(to_bytes(o.data(), 32));
    return res;
  });
  m.def("scrypt_1024_1_1", [](const py::bytes& h) {
    std::string s = need(h, 80, "header"); uint8_t o[32];
    { py::gil_scoped_release r; scrypt_1024_1_1(reinterpret_cast<const uint8_t*>(s.data()), o); }
    return to_bytes(o, 32);
  });
  // Test hook: the miner's device-clock estimate (ClockBounds) over a sequence of (seen at, offset bound) pairs;
  // returns the estimate after each.
  m.def("_clock_bounds", [](double window, const std::vector<std::pair<double, double>>& samples) {
    ClockBounds cb(window);
    std::vector<double> out;
    for (const auto& s : samples) out.push_back(cb.add(s.first, s.second));
    return out;
  });
  // Test hook: the scrypt verifier's bounded queue (BoundedWorkQueue) flooded by a producer that never waits, with
  // a consumer hashing every item on the host. batch > 1 takes up to that many items per pop_many and hashes them in
  // one scrypt_1024_1_1_batch pass, as the GPU miner's verifier does (16); batch 1 pops and hashes one at a time.
  m.def("_work_queue_flood", [](size_t cap, size_t n, bool hash_each, size_t batch) {
    BoundedWorkQueue<std::array<uint8_t, 80>> q(cap);
    std::atomic<uint64_t> processed{0};
    uint64_t accepted = 0;
    {
      py::gil_scoped_release r;
      std::thread consumer([&] {
        if (batch > 1) {
          std::vector<std::array<uint8_t, 80>> items;
          std::vector<const uint8_t*> ip;
          std::vector<std::array<uint8_t, 32>> outs(batch);
          std::vector<uint8_t*> op;
          for (auto& o : outs) op.push_back(o.data());
          while (items.clear(), q.pop_many(&items, batch) > 0) {
            ip.clear();
            for (const auto& it : items) ip.push_back(it.data());
            if (hash_each) scrypt_1024_1_1_batch(int(items.size()), ip.data(), op.data());
            processed.fetch_add(items.size());
          }
          return;
        }
        std::array<uint8_t, 80> h;
        uint8_t out[32];
        while (q.pop(&h)) {
          if (hash_each) scrypt_1024_1_1(h.data(), out);
          processed.fetch_add(1);
        }
      });
      for (size_t i = 0; i < n; ++i) {
        std::array<uint8_t, 80> h{};
        std::memcpy(h.data() + 76, &i, 4);
        if (q.push(std::move(h))) ++accepted;
      }
      q.stop(~size_t(0));
      consumer.join();
    }
    py::dict d;
    d["accepted"] = accepted;
    d["refused"] = q.refused();
    d["peak"] = q.peak();
    d["processed"] = processed.load();
    return d;
  }, py::arg("cap"), py::arg("n"), py::arg("hash_each") = true, py::arg("batch") = 1);
  m.attr("X11_STAGES") = kX11StageCount;
  m.def("x11", [](const py::bytes& msg) {
    std::string s = msg; uint8_t o[32];
    { py::gil_scoped_release r; x11::x11(reinterpret_cast<const uint8_t*>(s.data()), s.size(), o, nullptr); }
    return to_bytes(o, 32);
  }, py::arg("msg"));
  m.def("x11_trace", [](const py::bytes& msg) {
    std::string s = msg; uint8_t o[32], t[64 * kX11StageCount];
    x11::x11(reinterpret_cast<const uint8_t*>(s.data()), s.size(), o, t);
    return to_bytes(t, sizeof t);
  }, py::arg("msg"), "The 11 intermediate 64-byte digests of the X11 chain, concatenated.");
  m.def("x11_stage", [](int i, const py::bytes& msg) {
    if (i < 0 || i >= kX11StageCount) throw std::invalid_argument("stage must be in [0, 11)");
    std::string s = msg; uint8_t o[64];
    x11::stage(i, reinterpret_cast<const uint8_t*>(s.data()), s.size(), o);
    return to_bytes(o, 64);
  }, py::arg("stage"), py::arg("msg"));
  m.def("x11_luffa_sbox_selfcheck", &x11::luffa_sbox_selfcheck);
  m.def(
      "sv2_scan",
      [](py::buffer b, uint32_t max_frame) {
        py::buffer_info info = b.request();
        if (info.itemsize != 1 || info.ndim != 1) throw std::invalid_argument("sv2_scan: need a contiguous byte buffer");
        const size_t n = (size_t)info.size;
        if (n > 0xFFFFFFFFull) throw std::invalid_argument("sv2_scan: buffer larger than 4 GiB");
        // Upper bound on frames in n bytes: every frame has a 6-byte header.
        std::vector<Sv2FrameRec> recs(n / kSv2HeaderSize + 1);
        size_t consumed = 0, k = 0;
        int status = kSv2Ok;
        {
          py::gil_scoped_release nogil;
          k = sv2_scan(static_cast<const uint8_t*>(info.ptr), n, max_frame, recs.data(), recs.size(), &consumed,
                       &status);
        }
        py::list frames(k);
        for (size_t i = 0; i < k; ++i) {
          const Sv2FrameRec& r = recs[i];
          frames[i] = py::make_tuple(r.extension_type, r.msg_type, r.offset, r.length);
        }
        return py::make_tuple(frames, consumed, status);
      },
      py::arg("buf"), py::arg("max_frame"),
      "Split complete SV2 frames: ([(extension_type, msg_type, payload_offset, payload_length)], consumed, status)");
  m.def("cpu_scan_sha256d", [](const py::bytes& h, const py::bytes& t, uint32_t start, uint64_t count) {
    std::string hs = need(h, 80, "header"), ts = need(t, 32, "target");
    std::vector<uint32_t> hits;
    {
      py::gil_scoped_release r;
      hits = cpu_scan_sha256d(reinterpret_cast<const uint8_t*>(hs.data()), reinterpret_cast<const uint8_t*>(ts.data()),
                              start, count);
    }
    return hits;
  }, py::arg("header"), py::arg("target"), py::arg("start"), py::arg("count"));
  m.def("cpu_scan_method", &cpu_scan_method);
  // A/B hook: the CPU scan with a given number of nonces in flight per step (1..4 SHA-NI chains, 16 AVX-512).
  m.def("_cpu_scan_lanes", [](int lanes, const py::bytes& h, const py::bytes& t, uint32_t start, uint64_t count) {
    std::string hs = need(h, 80, "header"), ts = need(t, 32, "target");
    std::vector<uint32_t> hits;
    {
      py::gil_scoped_release r;
      hits = cpu_scan_sha256d_lanes(lanes, reinterpret_cast<const uint8_t*>(hs.data()),
                                    reinterpret_cast<const uint8_t*>(ts.data()), start, count);
    }
    return hits;
  });
  m.def("merkle_root", [](const py::dict& job, uint64_t en2) {
    auto j = make_job(job); uint8_t root[32];
    merkle_root_from_coinbase(*j, en2, root);
    return to_bytes(root, 32);
  });
  m.def("variant_header", [](const py::dict& job, uint64_t v) {
    auto j = make_job(job);
    uint8_t hdr[80]; uint32_t ver, nt; uint64_t en2;
    j->variant_header(v, hdr, &ver, &nt, &en2);
    return py::make_tuple(to_bytes(hdr, 80), ver, nt, en2);
  });
  m.def("variant_space", [](const py::dict& job) { return make_job(job)->variant_space(); });

  // Kernel parameter blocks are returned as opaque bytes and passed back in.
  m.def("sha256d_prepare", [](const py::bytes& h, const py::bytes& t) {
    std::string hs = need(h, 80, "header"), ts = need(t, 32, "target");
    Sha256dParams p;
    sha256d_prepare(reinterpret_cast<const uint8_t*>(hs.data()), reinterpret_cast<const uint8_t*>(ts.data()), &p);
    return py::bytes(reinterpret_cast<const char*>(&p), sizeof p);
  });
  m.attr("SHA256D_MAX_K") = kSha256dMaxK;
  {
    py::list ks;
    for (int k = 2; k <= kSha256dMaxK; ++k)
      if (sha256d_k_floor(k) == k) ks.append(k);
    m.attr("SHA256D_K_VALUES") = py::tuple(ks);
  }
  m.def("sha256d_prepare_k", [](const py::list& headers, const py::bytes& t) {
    std::string ts = need(t, 32, "target");
    std::vector<std::string> hs;
    for (auto& h : headers) hs.push_back(need(h.cast<py::bytes>(), 80, "header"));
    std::vector<const uint8_t*> ptrs;
    for (auto& h : hs) ptrs.push_back(reinterpret_cast<const uint8_t*>(h.data()));
    Sha256dParamsK p;
    if (!sha256d_prepare_k(ptrs.data(), (int)ptrs.size(), reinterpret_cast<const uint8_t*>(ts.data()), &p))
      throw std::invalid_argument("need K headers (K in SHA256D_K_VALUES) with identical bytes 64..75");
    return py::bytes(reinterpret_cast<const char*>(&p), sizeof p);
  }, py::arg("headers"), py::arg("target"));
  m.attr("SHA256D_V_GROUP") = kSha256dVGroup;
  m.attr("SHA256D_V2_GROUP") = kSha256dV2Group;
  m.def("sha256d_prepare_v", [](const py::list& headers, const py::bytes& t) {
    std::string ts = need(t, 32, "target");
    std::vector<std::string> hs;
    for (auto& h : headers) hs.push_back(need(h.cast<py::bytes>(), 80, "header"));
    std::vector<const uint8_t*> ptrs;
    for (auto& h : hs) ptrs.push_back(reinterpret_cast<const uint8_t*>(h.data()));
    Sha256dParamsV p;
    std::vector<Sha256dVariant> vars(hs.size());
    if (!sha256d_prepare_v(ptrs.data(), (int)ptrs.size(), reinterpret_cast<const uint8_t*>(ts.data()), &p, vars.data()))
      throw std::invalid_argument("need a positive multiple of 64 headers with identical bytes 64..75");
    return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&p), sizeof p),
                          py::bytes(reinterpret_cast<const char*>(vars.data()), vars.size() * sizeof(Sha256dVariant)));
  }, py::arg("headers"), py::arg("target"));
  m.def("scrypt_prepare", [](const py::bytes& h, const py::bytes& t) {
    std::string hs = need(h, 80, "header"), ts = need(t, 32, "target");
    ScryptParams p;
    scrypt_prepare(reinterpret_cast<const uint8_t*>(hs.data()), reinterpret_cast<const uint8_t*>(ts.data()), &p);
    return py::bytes(reinterpret_cast<const char*>(&p), sizeof p);
  });

  m.def("x11_prepare", [](const py::bytes& h, const py::bytes& t) {
    std::string hs = need(h, 80, "header"), ts = need(t, 32, "target");
    X11Params p;
    x11_prepare(reinterpret_cast<const uint8_t*>(hs.data()), reinterpret_cast<const uint8_t*>(ts.data()), &p);
    return py::bytes(reinterpret_cast<const char*>(&p), sizeof p);
  });

  // roctx ranges for Python-side spans (node collectives, share submit, bench steps): SURVEY §5.1.
  m.def("trace_push", [](const std::string& name) { trace_push(name.c_str()); });
  m.def("trace_pop", [] { trace_pop(); });
  m.def("trace_mark", [](const std::string& name) { trace_mark(name.c_str()); });
  m.def("gpu_device_count", &gpu_device_count);
  m.def("gpu_arch_name", &gpu_arch_name);
  m.def("gpu_cu_count", &gpu_cu_count);
  m.def("scrypt_scratch_bytes", &scrypt_scratch_bytes);
  // test hook: the /proc/self/maps check behind the CPU-stored abort word (GpuMiner host_abort)
  m.def("maps_range_writable", [](const std::string& maps, uint64_t lo, uint64_t hi) {
    return maps_range_writable(maps, uintptr_t(lo), uintptr_t(hi));
  });
  m.def("launch_sha256d", [](const py::bytes& params, uint32_t base, uint64_t count, uintptr_t out, uint32_t cap,
                             int grid, uintptr_t stream) {
    std::string ps = need(params, sizeof(Sha256dParams), "params");
    Sha256dParams p; std::memcpy(&p, ps.data(), sizeof p);
    if (count == 0 || count > (1ull << 32)) throw std::invalid_argument("count must be in [1, 2^32]");
    if (grid <= 0 || out == 0) throw std::invalid_argument("bad grid / out");
    py_launch_sha256d(p, base, count, out, cap, grid, stream);
  }, py::arg("params"), py::arg("base"), py::arg("count"), py::arg("out"), py::arg("cap"), py::arg("grid"),
     py::arg("stream"));
  m.def("launch_sha256d_k", [](const py::bytes& params, uint32_t base, uint64_t count, uintptr_t out, uint32_t cap,
                               int grid, uintptr_t stream) {
    std::string ps = need(params, sizeof(Sha256dParamsK), "params");
    Sha256dParamsK p; std::memcpy(&p, ps.data(), sizeof p);
    if (p.k < 2 || p.k > kSha256dMaxK) throw std::invalid_argument("bad K");
    if (count == 0 || count > (1ull << 32)) throw std::invalid_argument("count must be in [1, 2^32]");
    if (grid <= 0 || out == 0) throw std::invalid_argument("bad grid / out");
    py_launch_sha256d_k(p, base, count, out, cap, grid, stream);
  }, py::arg("params"), py::arg("base"), py::arg("count"), py::arg("out"), py::arg("cap"), py::arg("grid"),
     py::arg("stream"));
  m.def("launch_sha256d_v", [](const py::bytes& params, uintptr_t vars, uint32_t base, uint64_t count, uintptr_t out,
                               uint32_t cap, int grid, uintptr_t stream, bool occupancy8, int block, int chains) {
    std::string ps = need(params, sizeof(Sha256dParamsV), "params");
    Sha256dParamsV p; std::memcpy(&p, ps.data(), sizeof p);
    p.occupancy8 = occupancy8 ? 1u : 0u;
    if (p.groups == 0 || count == 0 || count > (1ull << 32)) throw std::invalid_argument("bad groups / count");
    if (block != 64 && block != 256) throw std::invalid_argument("block must be 64 or 256 threads");
    if (chains < 1 || chains > 4) throw std::invalid_argument("chains must be 1..4");
    if (p.groups % uint32_t(chains) != 0)
      throw std::invalid_argument("chains variants per lane need a multiple of 64 * chains variants");
    if (grid <= 0 || (uint64_t(grid) * uint32_t(block / 64)) % (p.groups / uint32_t(chains)) != 0 || vars == 0 || out == 0)
      throw std::invalid_argument("the wave count must be a multiple of the variant groups; vars/out must be set");
    py_launch_sha256d_v(p, vars, base, count, out, cap, grid, stream, block, chains);
  }, py::arg("params"), py::arg("vars"), py::arg("base"), py::arg("count"), py::arg("out"), py::arg("cap"),
     py::arg("grid"), py::arg("stream"), py::arg("occupancy8") = false, py::arg("block") = 256, py::arg("chains") = 1);
  m.def("launch_scrypt", [](const py::bytes& params, uint32_t base, uint32_t count, uintptr_t xbuf, uintptr_t scratch,
                            int gap, uintptr_t out, uint32_t cap, int grid, uintptr_t stream) {
    std::string ps = need(params, sizeof(ScryptParams), "params");
    ScryptParams p; std::memcpy(&p, ps.data(), sizeof p);
    if (gap != 1 && gap != 2 && gap != 4 && gap != kScryptCoop && gap != kScryptLaneW8 && gap != kScryptCoop2 &&
        gap != kScryptCoopSplit)
      throw std::invalid_argument("gap must be 1, 2, 4, SCRYPT_COOP or SCRYPT_LANE_W8");
    if (grid <= 0 || out == 0 || xbuf == 0 || scratch == 0 || count == 0) throw std::invalid_argument("bad launch args");
    py_launch_scrypt(p, base, count, xbuf, scratch, gap, out, cap, grid, stream);
  }, py::arg("params"), py::arg("base"), py::arg("count"), py::arg("xbuf"), py::arg("scratch"), py::arg("gap"),
     py::arg("out"), py::arg("cap"), py::arg("grid"), py::arg("stream"));

  m.def("launch_x11_stage", [](const py::bytes& params, int stage, uint32_t base, uintptr_t H, uint32_t stride,
                               uint32_t n, uintptr_t out, uint32_t cap, uintptr_t stream) {
    std::string ps = need(params, sizeof(X11Params), "params");
    X11Params p; std::memcpy(&p, ps.data(), sizeof p);
    if (stage < 0 || stage >= kX11StageCount) throw std::invalid_argument("stage must be in [0, 11)");
    if (H == 0 || n == 0 || stride < n) throw std::invalid_argument("need H != 0, n > 0, stride >= n");
    py_launch_x11_stage(p, stage, base, H, stride, n, out, cap, stream);
  }, py::arg("params"), py::arg("stage"), py::arg("base"), py::arg("H"), py::arg("stride"), py::arg("n"),
     py::arg("out") = 0, py::arg("cap") = 0, py::arg("stream") = 0);
  m.def("launch_x11", [](const py::bytes& params, uint32_t base, uintptr_t H, uint32_t stride, uint32_t n,
                         uintptr_t out, uint32_t cap, uintptr_t stream) {
    std::string ps = need(params, sizeof(X11Params), "params");
    X11Params p; std::memcpy(&p, ps.data(), sizeof p);
    if (H == 0 || n == 0 || stride < n) throw std::invalid_argument("need H != 0, n > 0, stride >= n");
    py_launch_x11(p, base, H, stride, n, out, cap, stream);
  }, py::arg("params"), py::arg("base"), py::arg("H"), py::arg("stride"), py::arg("n"), py::arg("out") = 0,
     py::arg("cap") = 0, py::arg("stream") = 0);

  py::class_<MinerBase, std::shared_ptr<MinerBase>>(m, "Miner")
      .def("start", &MinerBase::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &MinerBase::stop, py::call_guard<py::gil_scoped_release>())
      .def("set_job", [](MinerBase& self, py::object job) {
        if (job.is_none()) { py::gil_scoped_release r; self.set_job(nullptr); return; }
        auto j = make_job(job.cast<py::dict>());
        py::gil_scoped_release r;
        self.set_job(j);
      })
      .def("poll", [](MinerBase& self, size_t max) {
        std::vector<ShareRecord> v;
        { py::gil_scoped_release r; v = self.poll(max); }
        return shares_to_list(std::move(v));
      }, py::arg("max") = 256)
      .def("stats", [](MinerBase& self) { return stats_to_dict(self.stats()); })
      .def("share_fd", &MinerBase::share_fd,
           "eventfd that becomes readable when shares are queued (read 8 bytes to reset, then poll())")
      .def_property_readonly("device_id", &MinerBase::device_id);

  py::class_<GpuMiner, MinerBase, std::shared_ptr<GpuMiner>>(m, "GpuMiner")
      .def(py::init<int, std::string, uint64_t, int, size_t, int>(), py::arg("device"), py::arg("device_id"),
           py::arg("batch_nonces") = (1ull << 32), py::arg("grid") = 2048, py::arg("queue_cap") = 1024,
           py::arg("sha_variants") = 128);
  py::class_<CpuMiner, MinerBase, std::shared_ptr<CpuMiner>>(m, "CpuMiner")
      .def(py::init<int, std::string, size_t>(), py::arg("threads"), py::arg("device_id") = "cpu-0",
           py::arg("queue_cap") = 1024);

  m.attr("SHA256D_PARAMS_SIZE") = sizeof(Sha256dParams);
  m.attr("SHA256D_V_PARAMS_SIZE") = sizeof(Sha256dParamsV);
  m.attr("SCRYPT_PARAMS_SIZE") = sizeof(ScryptParams);
}
