// Native RCCL data plane of the multi-GPU node: R1 (job broadcast), R2 (share gather), R3 (counters), SURVEY §7.1
// ("the RCCL comm layer (R1-R3)" in C++) and §5.8 (one comm stream per GPU, pinned host buffers on the pool side).
//
// One RcclComm per rank process and process-group generation (otedama_amd/parallel/rcclcomm.py owns the unique-id
// exchange through the node's store and the generations). Design points, each measured on the MI355X
// (profiles/r5/d_comm_ab):
//   * every op is ONE chain on one high-priority HIP stream: pinned host staging -> device, the RCCL collective,
//     device -> pinned host, an event. The GPU is saturated by the sibling device process's mining grid; a kernel or
//     blit of this process on a normal-priority queue waited behind it for a CU slot (R2 4.5 ms p50 with the copies
//     on the default stream, 1.9 ms with everything on high-priority streams);
//   * the communicator is non-blocking (ncclConfig_t.blocking = 0): init and every op are polled against a deadline
//     with the GIL released, so a dead peer never hangs the caller; ncclCommAbort tears a broken group down at once;
//   * no torch in the process: the node's rank processes import only this module and the native miner bindings
//     (start-up: `import torch` was ~1.45 s of a rank's 1.8 s to its process group, profiles/r5/c_node_rehearsal);
//   * device-resident ops (`*_dev`): the collective reads and writes device memory the caller owns (bench.py's hit
//     slots, the comm section's 256 MiB bus-bandwidth buffer) and is enqueued on the caller's HIP stream, so nothing
//     is staged through the host and the traffic is GPU to GPU over xGMI. Every op of a communicator, staged or not,
//     is ordered on the device after the previous one (an event hand-off between streams), so ranks that issue the
//     same op sequence run it in the same order whatever streams they used.
//
// The reference has no collective layer; its fan-out / fan-in are Go channels
// (internal/engine/fanin.go:22-58), which never block a producer: the deadlines here keep that property.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <pybind11/pybind11.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace py = pybind11;

namespace {

struct RcclTimeout : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Poll-wait: yield for the first 2 ms (a small collective completes in ~0.1-0.2 ms once every rank is in it), then
// 100 us sleeps up to the deadline. `ready` returns 1 (done), 0 (not yet) or throws.
template <class F>
void wait_until(F ready, double timeout_s, const char* what) {
  const double t0 = now_s(), end = t0 + timeout_s, spin_until = t0 + 0.002;
  for (;;) {
    if (ready()) return;
    const double t = now_s();
    if (t > end) throw RcclTimeout(std::string(what) + " did not finish in " + std::to_string(timeout_s) + " s");
    if (t < spin_until) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}

class RcclComm {
 public:
  RcclComm(int device, int nranks, int rank, const std::string& uid, double timeout_s)
      : device_(device), nranks_(nranks), rank_(rank) {
    if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("unique id must be 128 bytes");
    if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("bad rank / nranks");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
    hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority");
    hip_check(hipEventCreateWithFlags(&done_, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&order_, hipEventDisableTiming), "hipEventCreate");
    ncclUniqueId id;
    std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;
      r = ncclCommInitRankConfig(&comm_, nranks_, id, rank_, &cfg);
      if (r == ncclSuccess || r == ncclInProgress) {
        try {
          wait_until([&] { return settled(); }, timeout_s, "ncclCommInitRankConfig");
          r = ncclSuccess;
        } catch (...) {
          abort_nogil();
          release();
          throw;
        }
      }
    }
    if (r != ncclSuccess) {
      release();
      throw std::runtime_error(std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
    }
  }
  ~RcclComm() {
    abort_nogil();
    release();
  }
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int nranks() const { return nranks_; }
  int rank() const { return rank_; }
  int device() const { return device_; }
  bool alive() const { return comm_ != nullptr; }
  uint64_t ops() const { return ops_; }

  // R1: root's `data` (nbytes) to every rank; returns the nbytes every rank now holds.
  py::bytes broadcast(const std::string& data, size_t nbytes, int root, double timeout_s) {
    if (rank_ == root && data.size() != nbytes) throw std::invalid_argument("root's data must be nbytes long");
    usable();
    ensure(nbytes, nbytes);
    std::string out(nbytes, '\0');
    {
      py::gil_scoped_release nogil;
      if (rank_ == root) std::memcpy(host_, data.data(), nbytes);
      run(nbytes, nbytes, timeout_s, "broadcast",
          [&] { return ncclBroadcast(dev_, dev_, nbytes, ncclUint8, root, comm_, stream_); });
      std::memcpy(out.data(), host_, nbytes);
    }
    return py::bytes(out);
  }

  // R2 / R3: every rank's `mine` (same length everywhere), concatenated in rank order.
  py::bytes all_gather(const std::string& mine, double timeout_s) {
    const size_t n = mine.size(), total = n * size_t(nranks_);
    usable();
    ensure(n, total);
    std::string out(total, '\0');
    {
      py::gil_scoped_release nogil;
      // in place: rank r's contribution sits at offset r * n of the receive buffer
      std::memcpy(static_cast<char*>(host_) + size_t(rank_) * n, mine.data(), n);
      run(n, total, timeout_s, "all_gather", [&] {
        return ncclAllGather(static_cast<char*>(dev_) + size_t(rank_) * n, dev_, n, ncclUint8, comm_, stream_);
      }, size_t(rank_) * n);
      std::memcpy(out.data(), host_, total);
    }
    return py::bytes(out);
  }

  // R3: element-wise sum (or max) of `data` across ranks; dtype "i64" or "f64".
  py::bytes all_reduce(const std::string& data, const std::string& dtype, const std::string& op, double timeout_s) {
    const ncclDataType_t t = dtype == "f64" ? ncclFloat64 : ncclInt64;
    if (dtype != "f64" && dtype != "i64") throw std::invalid_argument("dtype must be i64 or f64");
    const ncclRedOp_t o = op == "max" ? ncclMax : ncclSum;
    if (op != "max" && op != "sum") throw std::invalid_argument("op must be sum or max");
    if (data.size() % 8) throw std::invalid_argument("data must be whole 8-byte elements");
    const size_t n = data.size();
    usable();
    ensure(n, n);
    std::string out(n, '\0');
    {
      py::gil_scoped_release nogil;
      std::memcpy(host_, data.data(), n);
      run(n, n, timeout_s, "all_reduce",
          [&] { return ncclAllReduce(dev_, dev_, n / 8, t, o, comm_, stream_); });
      std::memcpy(out.data(), host_, n);
    }
    return py::bytes(out);
  }

  // Device-resident forms: pointers to device memory of this comm's GPU (torch's data_ptr()), enqueued on `stream`
  // (a hipStream_t as an integer, torch's Stream.cuda_stream; 0 = the comm's own stream). They return once the op is
  // enqueued (the non-blocking communicator settled); completion is the caller's, through its stream.
  void all_gather_dev(uintptr_t send, uintptr_t recv, size_t nbytes, uintptr_t stream, double timeout_s) {
    enqueue(stream, timeout_s, "all_gather_dev", [&](hipStream_t s) {
      return ncclAllGather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), nbytes, ncclUint8, comm_,
                           s);
    });
  }
  void broadcast_dev(uintptr_t buf, size_t nbytes, int root, uintptr_t stream, double timeout_s) {
    if (root < 0 || root >= nranks_) throw std::invalid_argument("bad root");
    enqueue(stream, timeout_s, "broadcast_dev", [&](hipStream_t s) {
      return ncclBroadcast(reinterpret_cast<const void*>(buf), reinterpret_cast<void*>(buf), nbytes, ncclUint8, root,
                           comm_, s);
    });
  }
  void all_reduce_dev(uintptr_t buf, size_t count, const std::string& dtype, const std::string& op, uintptr_t stream,
                      double timeout_s) {
    if (dtype != "f64" && dtype != "i64") throw std::invalid_argument("dtype must be i64 or f64");
    if (op != "max" && op != "sum") throw std::invalid_argument("op must be sum or max");
    const ncclDataType_t t = dtype == "f64" ? ncclFloat64 : ncclInt64;
    const ncclRedOp_t o = op == "max" ? ncclMax : ncclSum;
    enqueue(stream, timeout_s, "all_reduce_dev", [&](hipStream_t s) {
      return ncclAllReduce(reinterpret_cast<const void*>(buf), reinterpret_cast<void*>(buf), count, t, o, comm_, s);
    });
  }

  // Tear the communicator down at once (a peer died, or a new generation is formed): ncclCommAbort never waits for
  // the peers. Idempotent.
  void abort() {
    py::gil_scoped_release nogil;
    abort_nogil();
  }

 private:
  void abort_nogil() {
    if (comm_ == nullptr) return;
    (void)ncclCommAbort(comm_);
    comm_ = nullptr;
  }

  // An op may start: the communicator exists and no earlier op timed out. Checked before anything touches the staging
  // buffers (ensure() may free them, and a timed-out op may still be queued on them: ADVICE r5).
  void usable() const {
    if (comm_ == nullptr) throw std::runtime_error("rccl: communicator aborted");
    if (broken_) throw std::runtime_error("rccl: an earlier op timed out; abort this communicator and re-form");
  }

  // Device order across streams: `s` waits for the previous op of this communicator when that op went to another
  // stream; the op about to be enqueued on `s` is recorded by after().
  void order_on(hipStream_t s) {
    if (last_stream_ != nullptr && last_stream_ != s) hip_check(hipStreamWaitEvent(s, order_, 0), "hipStreamWaitEvent");
  }
  void after(hipStream_t s) {
    hip_check(hipEventRecord(order_, s), "hipEventRecord");
    last_stream_ = s;
  }

  template <class Start>
  void enqueue(uintptr_t stream, double timeout_s, const char* what, Start start) {
    usable();
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : stream_;
    py::gil_scoped_release nogil;
    hip_check(hipSetDevice(device_), "hipSetDevice");
    order_on(s);
    const ncclResult_t r = start(s);
    if (r != ncclSuccess && r != ncclInProgress)
      throw std::runtime_error(std::string("rccl ") + what + ": " + ncclGetErrorString(r));
    try {
      if (r == ncclInProgress) wait_until([&] { return settled(); }, timeout_s, what);
    } catch (...) {
      broken_ = true;
      throw;
    }
    after(s);
    ++ops_;
  }

  // The communicator's asynchronous state: 1 = settled, 0 = in progress; throws on an error.
  int settled() {
    ncclResult_t st = ncclSuccess;
    const ncclResult_t q = ncclCommGetAsyncError(comm_, &st);
    if (q != ncclSuccess) throw std::runtime_error(std::string("ncclCommGetAsyncError: ") + ncclGetErrorString(q));
    if (st == ncclInProgress) return 0;
    if (st != ncclSuccess) throw std::runtime_error(std::string("rccl: ") + ncclGetErrorString(st));
    return 1;
  }

  void ensure(size_t in_bytes, size_t out_bytes) {
    const size_t need = std::max(in_bytes, out_bytes);
    if (need <= cap_) return;
    size_t cap = 64 << 10;
    while (cap < need) cap *= 2;
    hip_check(hipSetDevice(device_), "hipSetDevice");
    if (dev_) (void)hipFree(dev_);
    if (host_) (void)hipHostFree(host_);
    dev_ = nullptr;
    host_ = nullptr;
    cap_ = 0;
    hip_check(hipMalloc(&dev_, cap), "hipMalloc");
    hip_check(hipHostMalloc(&host_, cap, hipHostMallocDefault), "hipHostMalloc");
    cap_ = cap;
  }

  // One op, all on the comm stream: host_[in_off, in_off + in_bytes) (placed there by the caller) -> dev_ at the same
  // offset, the collective,
  // dev_[0, out_bytes) -> host_, then the event polled against the deadline (and the communicator's async error).
  template <class Start>
  void run(size_t in_bytes, size_t out_bytes, double timeout_s, const char* what, Start start, size_t in_off = 0) {
    // An op that timed out may still be queued on the stream (its peer never came): the next op would stage into
    // the buffers it reads and writes. Such a communicator only serves an abort (usable(), checked by the caller
    // before it staged anything).
    hip_check(hipSetDevice(device_), "hipSetDevice");
    char* h = static_cast<char*>(host_);
    char* d = static_cast<char*>(dev_);
    order_on(stream_);
    hip_check(hipMemcpyAsync(d + in_off, h + in_off, in_bytes, hipMemcpyHostToDevice, stream_), "hipMemcpyAsync H2D");
    ncclResult_t r = start();
    if (r != ncclSuccess && r != ncclInProgress)
      throw std::runtime_error(std::string("rccl ") + what + ": " + ncclGetErrorString(r));
    try {
      if (r == ncclInProgress) wait_until([&] { return settled(); }, timeout_s, what);  // non-blocking enqueue
      hip_check(hipMemcpyAsync(h, d, out_bytes, hipMemcpyDeviceToHost, stream_), "hipMemcpyAsync D2H");
      after(stream_);
      hip_check(hipEventRecord(done_, stream_), "hipEventRecord");
      wait_until([&] {
        const hipError_t q = hipEventQuery(done_);
        if (q == hipSuccess) return 1;
        if (q != hipErrorNotReady) hip_check(q, "hipEventQuery");
        settled();  // a failed peer surfaces here while the event never completes
        return 0;
      }, timeout_s, what);
    } catch (...) {
      broken_ = true;
      throw;
    }
    ++ops_;
  }

  void release() {
    if (dev_) (void)hipFree(dev_);
    if (host_) (void)hipHostFree(host_);
    if (done_) (void)hipEventDestroy(done_);
    if (order_) (void)hipEventDestroy(order_);
    if (stream_) (void)hipStreamDestroy(stream_);
    dev_ = host_ = nullptr;
    done_ = order_ = nullptr;
    last_stream_ = nullptr;
    stream_ = nullptr;
    cap_ = 0;
  }

  int device_, nranks_, rank_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t done_ = nullptr;
  hipEvent_t order_ = nullptr;      // recorded after every op, on the stream it went to
  hipStream_t last_stream_ = nullptr;
  void* dev_ = nullptr;
  void* host_ = nullptr;
  size_t cap_ = 0;
  uint64_t ops_ = 0;
  bool broken_ = false;
};

py::bytes unique_id() {
  ncclUniqueId id;
  ncclResult_t r;
  {
    py::gil_scoped_release nogil;
    r = ncclGetUniqueId(&id);
  }
  if (r != ncclSuccess) throw std::runtime_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

std::string version() {
  int v = 0;
  ncclGetVersion(&v);
  return std::to_string(v);
}

}  // namespace

PYBIND11_MODULE(_rccl, m) {
  m.doc() = "Native RCCL data plane of the otedama node (R1/R2/R3 on a high-priority HIP stream)";
  py::register_exception<RcclTimeout>(m, "RcclTimeout", PyExc_TimeoutError);
  m.def("unique_id", &unique_id, "ncclGetUniqueId: 128 bytes for the group's rank 0 to publish");
  m.def("version", &version);
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<int, int, int, const std::string&, double>(), py::arg("device"), py::arg("nranks"),
           py::arg("rank"), py::arg("unique_id"), py::arg("timeout_s"))
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("alive", &RcclComm::alive)
      .def_property_readonly("ops", &RcclComm::ops)
      .def("broadcast", &RcclComm::broadcast, py::arg("data"), py::arg("nbytes"), py::arg("root"),
           py::arg("timeout_s"))
      .def("all_gather", &RcclComm::all_gather, py::arg("mine"), py::arg("timeout_s"))
      .def("all_reduce", &RcclComm::all_reduce, py::arg("data"), py::arg("dtype"), py::arg("op"),
           py::arg("timeout_s"))
      .def("all_gather_dev", &RcclComm::all_gather_dev, py::arg("send"), py::arg("recv"), py::arg("nbytes"),
           py::arg("stream"), py::arg("timeout_s"))
      .def("broadcast_dev", &RcclComm::broadcast_dev, py::arg("buf"), py::arg("nbytes"), py::arg("root"),
           py::arg("stream"), py::arg("timeout_s"))
      .def("all_reduce_dev", &RcclComm::all_reduce_dev, py::arg("buf"), py::arg("count"), py::arg("dtype"),
           py::arg("op"), py::arg("stream"), py::arg("timeout_s"))
      .def_property_readonly("device", [](const RcclComm& c) { return c.device(); })
      .def("abort", &RcclComm::abort);
}
