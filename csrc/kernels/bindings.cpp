// pybind11 bindings of the gfx950 kernels and HIP runtime helpers:
// module ddl_amd._ddl_hip.
//
// Every device/host buffer crosses this boundary as a raw address (int) and
// every launch takes an explicit hipStream_t handle (torch.cuda.Stream's
// .cuda_stream); dtype/shape validation lives in ddl_amd/ops/kernels.py.
// Keeping torch headers out of this TU keeps one HIP runtime (torch/lib's,
// linked by path) and no libtorch ABI coupling.
#include <dlfcn.h>
#include <errno.h>
#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "launch.h"
#include "engine.h"
#include "stager.h"

namespace py = pybind11;

namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

py::dict staged_dict(const ddl::StagedInfo& i) {
  py::dict d;
  d["window"] = i.window;
  d["buffer"] = i.buffer;
  d["producer"] = i.producer;
  d["slot"] = i.slot;
  d["seq"] = i.seq;
  d["used_bytes"] = i.used_bytes;
  d["tag"] = py::make_tuple(i.tag[0], i.tag[1], i.tag[2], i.tag[3]);
  d["t_ready_host"] = i.t_ready_host;
  d["meta"] = py::tuple(py::cast(i.meta));
  return d;
}

void check_rc(int rc, const char* what) {
  if (rc == 0) return;
  if (rc > 0) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(static_cast<hipError_t>(rc)));
  throw std::invalid_argument(std::string(what) + ": unsupported arguments (code " + std::to_string(rc) + ")");
}

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

template <typename T>
T* as_ptr(uintptr_t a) {
  return reinterpret_cast<T*>(a);
}

ddl::FeistelKeys make_keys(const std::vector<uint64_t>& k, uint64_t n, uint32_t half_bits) {
  if (k.size() != ddl::kFeistelRounds) throw std::invalid_argument("feistel: need 6 round keys");
  ddl::FeistelKeys f{};
  for (int i = 0; i < ddl::kFeistelRounds; ++i) f.k[i] = k[i];
  f.n = n;
  f.half_bits = half_bits;
  return f;
}

ddl::RowIndex make_index(int mode, uintptr_t idx, int64_t base, const std::vector<uint64_t>& keys, uint64_t n,
                         uint32_t half_bits) {
  ddl::RowIndex ri{};
  ri.mode = mode;
  ri.idx = as_ptr<const int64_t>(idx);
  ri.base = base;
  if (mode == 1 && !idx) throw std::invalid_argument("index mode 1 needs an index vector");
  if (mode == 2) ri.keys = make_keys(keys, n, half_bits);
  return ri;
}

ddl::Affine make_affine(const std::vector<float>& scale, const std::vector<float>& bias, int64_t plane) {
  ddl::Affine a{};
  if (scale.empty()) return a;
  if (scale.size() != bias.size() || scale.size() > static_cast<size_t>(ddl::kMaxAffineChannels))
    throw std::invalid_argument("affine: 1..16 channels");
  if (plane <= 0) throw std::invalid_argument("affine: plane must be > 0");
  for (size_t i = 0; i < scale.size(); ++i) {
    a.scale[i] = scale[i];
    a.bias[i] = bias[i];
  }
  a.channels = static_cast<int32_t>(scale.size());
  a.plane = plane;
  a.enabled = 1;
  return a;
}

// Host callback run by the HIP runtime once every prior op on the stream has
// retired: hands a shm slot back to its producer (state store + futex wake).
struct ReleaseReq {
  std::atomic<uint32_t>* word;
  uint32_t value;
};

void release_cb(void* p) {
  auto* r = static_cast<ReleaseReq*>(p);
  r->word->store(r->value, std::memory_order_release);
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(r->word), FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
  delete r;
}

}  // namespace

PYBIND11_MODULE(_ddl_hip, m) {
  m.doc() = "ddl_amd gfx950 HIP kernels (permute/gather, collate, pad/pack, checksum) and HIP runtime helpers";

  m.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("arch_name", [](int dev) {
    hipDeviceProp_t p;
    check(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
    return std::string(p.gcnArchName);
  });

  // ---------------------------------------------------------------- memory
  m.def(
      "host_register",
      [](uintptr_t addr, uint64_t bytes, bool mapped) {
        unsigned flags = hipHostRegisterPortable | (mapped ? hipHostRegisterMapped : 0u);
        py::gil_scoped_release nogil;
        check(hipHostRegister(as_ptr<void>(addr), bytes, flags), "hipHostRegister");
      },
      py::arg("addr"), py::arg("bytes"), py::arg("mapped") = true);
  m.def("host_unregister", [](uintptr_t addr) { check(hipHostUnregister(as_ptr<void>(addr)), "hipHostUnregister"); });
  m.def("host_device_pointer", [](uintptr_t addr) {
    void* d = nullptr;
    check(hipHostGetDevicePointer(&d, as_ptr<void>(addr), 0), "hipHostGetDevicePointer");
    return reinterpret_cast<uintptr_t>(d);
  });
  m.def(
      "dma_gather_rows",
      [](uintptr_t dst, uintptr_t src, uint64_t row_bytes, uintptr_t idx_ptr, int64_t n, int64_t src_rows,
         uintptr_t stream, bool batched) {
        // SDMA gather: row idx[i] of the (pinned, registered) host source -> row i of dst, as n copies in ONE
        // hipMemcpyBatchAsync (batched) or n hipMemcpyAsync calls; runs of consecutive rows become one copy.
        // Returns the host ns spent enqueueing.
        const auto t0 = std::chrono::steady_clock::now();
        const auto* idx = reinterpret_cast<const int64_t*>(idx_ptr);
        for (int64_t i = 0; i < n; ++i)  // an out-of-range row would DMA from unrelated host memory
          if (idx[i] < 0 || idx[i] >= src_rows) throw std::out_of_range("dma_gather_rows: row index out of range");
        std::vector<void*> dsts, srcs;
        std::vector<size_t> sizes;
        dsts.reserve(static_cast<size_t>(n));
        srcs.reserve(static_cast<size_t>(n));
        sizes.reserve(static_cast<size_t>(n));
        auto* d = reinterpret_cast<char*>(dst);
        const auto* sb = reinterpret_cast<const char*>(src);
        for (int64_t i = 0; i < n;) {
          int64_t j = i + 1;
          while (j < n && idx[j] == idx[j - 1] + 1) ++j;
          dsts.push_back(d + static_cast<uint64_t>(i) * row_bytes);
          srcs.push_back(const_cast<char*>(sb) + static_cast<uint64_t>(idx[i]) * row_bytes);
          sizes.push_back(static_cast<size_t>(j - i) * row_bytes);
          i = j;
        }
        py::gil_scoped_release nogil;
        // hipMemcpyBatchAsync is newer than the HIP runtime torch ships (ROCm 7.0): looked up at run time
        using BatchFn = hipError_t (*)(void**, void**, size_t*, size_t, hipMemcpyAttributes*, size_t*, size_t,
                                       size_t*, hipStream_t);
        static const auto batch_fn = reinterpret_cast<BatchFn>(dlsym(RTLD_DEFAULT, "hipMemcpyBatchAsync"));
        if (batched && batch_fn != nullptr) {
          size_t fail = 0;
          check(batch_fn(dsts.data(), srcs.data(), sizes.data(), dsts.size(), nullptr, nullptr, 0, &fail,
                         as_stream(stream)),
                "hipMemcpyBatchAsync");
        } else {
          for (size_t k = 0; k < dsts.size(); ++k)
            check(hipMemcpyAsync(dsts[k], srcs[k], sizes[k], hipMemcpyHostToDevice, as_stream(stream)),
                  "hipMemcpyAsync");
        }
        return static_cast<int64_t>(
            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
      },
      py::arg("dst"), py::arg("src"), py::arg("row_bytes"), py::arg("idx"), py::arg("n"), py::arg("src_rows"),
      py::arg("stream"), py::arg("batched") = true);
  m.def("has_memcpy_batch", [] { return dlsym(RTLD_DEFAULT, "hipMemcpyBatchAsync") != nullptr; });
  m.def("pointer_is_host_registered", [](uintptr_t addr) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, as_ptr<void>(addr)) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return a.type == hipMemoryTypeHost;
  });
  m.def(
      "memcpy_h2d",
      [](uintptr_t dst, uintptr_t src, uint64_t bytes, uintptr_t stream) {
        check(hipMemcpyAsync(as_ptr<void>(dst), as_ptr<const void>(src), bytes, hipMemcpyHostToDevice,
                             as_stream(stream)),
              "hipMemcpyAsync(H2D)");
      },
      py::arg("dst"), py::arg("src"), py::arg("bytes"), py::arg("stream"));
  m.def(
      "memcpy_d2h",
      [](uintptr_t dst, uintptr_t src, uint64_t bytes, uintptr_t stream) {
        check(hipMemcpyAsync(as_ptr<void>(dst), as_ptr<const void>(src), bytes, hipMemcpyDeviceToHost,
                             as_stream(stream)),
              "hipMemcpyAsync(D2H)");
      },
      py::arg("dst"), py::arg("src"), py::arg("bytes"), py::arg("stream"));
  m.def(
      "memcpy_d2d",
      [](uintptr_t dst, uintptr_t src, uint64_t bytes, uintptr_t stream) {
        check(hipMemcpyAsync(as_ptr<void>(dst), as_ptr<const void>(src), bytes, hipMemcpyDeviceToDevice,
                             as_stream(stream)),
              "hipMemcpyAsync(D2D)");
      },
      py::arg("dst"), py::arg("src"), py::arg("bytes"), py::arg("stream"));
  m.def(
      "enqueue_release",
      [](uintptr_t state_word, uint32_t value, uintptr_t stream) {
        auto* r = new ReleaseReq{as_ptr<std::atomic<uint32_t>>(state_word), value};
        hipError_t e = hipLaunchHostFunc(as_stream(stream), release_cb, r);
        if (e != hipSuccess) {
          delete r;
          check(e, "hipLaunchHostFunc");
        }
      },
      py::arg("state_word"), py::arg("value"), py::arg("stream"),
      "Store `value` into the shm slot state word (+ futex wake) once the stream reaches this point.");

  // ---------------------------------------------------------- native stager
  m.attr("ARENA_ABI") = ddl::arena_abi();
  py::class_<ddl::NativeStager>(m, "NativeStager")
      .def(py::init([](uintptr_t arena, int32_t n_producers, int32_t n_slots, int64_t first, int64_t total,
                       std::vector<uintptr_t> buffers, uint64_t buffer_bytes, uintptr_t copy_stream, int device,
                       std::vector<int32_t> peer_pids, int64_t timeout_ms, std::vector<uintptr_t> ready,
                       std::vector<uintptr_t> copy_done, bool post_copy, int64_t meta_bytes, uintptr_t copy_stream2,
                       bool direct_dma, bool copy_timing) {
             std::vector<void*> bufs;
             for (auto b : buffers) bufs.push_back(as_ptr<void>(b));
             std::vector<hipEvent_t> rd, cd;
             for (auto e : ready) rd.push_back(reinterpret_cast<hipEvent_t>(e));
             for (auto e : copy_done) cd.push_back(reinterpret_cast<hipEvent_t>(e));
             return std::make_unique<ddl::NativeStager>(
                 reinterpret_cast<const ddl::Arena*>(arena), n_producers, n_slots, first, total, std::move(bufs),
                 buffer_bytes, as_stream(copy_stream), device, std::move(peer_pids), timeout_ms, std::move(rd),
                 std::move(cd), post_copy, meta_bytes, as_stream(copy_stream2), direct_dma, copy_timing);
           }),
           py::arg("arena"), py::arg("n_producers"), py::arg("n_slots"), py::arg("first"), py::arg("total"),
           py::arg("buffers"), py::arg("buffer_bytes"), py::arg("copy_stream"), py::arg("device"),
           py::arg("peer_pids"), py::arg("timeout_ms"), py::arg("ready"), py::arg("copy_done"),
           py::arg("post_copy"), py::arg("meta_bytes") = 0, py::arg("copy_stream2") = 0,
           py::arg("direct_dma") = false, py::arg("copy_timing") = false)
      .def(
          "wait",
          [](ddl::NativeStager& st, int64_t w, int64_t timeout_ms) {
            ddl::StagedInfo info;
            int32_t fp = -1;
            int rc;
            {
              py::gil_scoped_release nogil;
              rc = st.wait(w, timeout_ms, &info, &fp);
            }
            return py::make_tuple(rc, fp, rc == 0 ? staged_dict(info) : py::dict());
          },
          py::arg("window"), py::arg("timeout_ms"),
          "(0, -1, info) once window w is staged, else (code, producer, {}): 1 shutdown, 2 timeout, 3 peer dead, "
          "4 peer failed, -1 internal error (see error())")
      .def(
          "peek",
          [](ddl::NativeStager& st, int64_t w) -> py::object {
            ddl::StagedInfo info;
            if (!st.peek(w, &info)) return py::none();
            return staged_dict(info);
          },
          py::arg("window"))
      .def(
          "release", [](ddl::NativeStager& st, int64_t w, uintptr_t ev) { st.release(w, reinterpret_cast<hipEvent_t>(ev)); },
          py::arg("window"), py::arg("free_event"))
      .def(
          "close",
          [](ddl::NativeStager& st) {
            py::gil_scoped_release nogil;
            st.close();
          })
      .def("error", &ddl::NativeStager::error)
      .def_property_readonly("bytes_h2d", &ddl::NativeStager::bytes_h2d)
      .def_property_readonly("windows_staged", &ddl::NativeStager::windows_staged)
      .def_property_readonly("windows_landed", &ddl::NativeStager::windows_landed)
      .def("settle", &ddl::NativeStager::settle, py::arg("timeout_ms") = 1000, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("bytes_landed", &ddl::NativeStager::bytes_landed)
      .def_property_readonly("wait_producer_s", &ddl::NativeStager::wait_producer_s)
      .def_property_readonly("free_waits", &ddl::NativeStager::free_waits)
      .def_property("free_on_host", &ddl::NativeStager::free_on_host, &ddl::NativeStager::set_free_on_host)
      .def_property("record_ready", &ddl::NativeStager::record_ready, &ddl::NativeStager::set_record_ready)
      .def_property_readonly("direct_dma", &ddl::NativeStager::direct_dma)
      .def_property_readonly("direct_dma_reason", &ddl::NativeStager::direct_dma_reason)
      .def_property_readonly("error_code", &ddl::NativeStager::error_code)
      .def("wait_copy", &ddl::NativeStager::wait_copy_window, py::arg("window"),
           py::call_guard<py::gil_scoped_release>(),
           "host wait for staged window w's copy, bounded by the stager's timeout: 0 landed, 2 timed out (the "
           "stager has failed: error()), 1 closed, -1 error")
      .def(
          "set_copy_timing", [](ddl::NativeStager& st, bool on) { return st.set_copy_timing(on); }, py::arg("on"),
          "device times for every direct-DMA copy (ROCr async-copy profiling: a process-wide switch, reference "
          "counted over stagers); False if ROCr refuses")
      .def_property_readonly("copy_timing", &ddl::NativeStager::copy_timing)
      .def("set_anchor_every", &ddl::NativeStager::set_anchor_every, py::arg("n"))
      .def_property_readonly("reanchors", &ddl::NativeStager::reanchors)
      .def("inject_stuck_copy", &ddl::NativeStager::inject_stuck_copy, py::arg("window"),
           "fault injection: window w's copy never reads as landed (its completion signal is armed one too high)")
      .def("inject_slow_retire", &ddl::NativeStager::inject_slow_retire, py::arg("extra_ms"),
           "fault injection: the retire thread waits extra_ms longer than the timeout (the consumer times out first)")
      .def_property_readonly("poisoned", &ddl::NativeStager::poisoned,
                             "a copy wait failed with copies pending: keep the ring and the arena alive")
      .def_property_readonly("leaked_signals", &ddl::NativeStager::leaked_signals)
      .def(
          "copies_between",
          [](const ddl::NativeStager& st, uint64_t t0, uint64_t t1) {
            const ddl::CopiesBetween c = st.copies_between(t0, t1);
            return py::make_tuple(c.windows, c.bytes, c.complete);
          },
          py::arg("t0_ns"), py::arg("t1_ns"),
          "(windows, bytes, complete) of H2D copies enqueued in [t0_ns, t1_ns] (CLOCK_MONOTONIC) that have "
          "retired; complete is False when older copy records were dropped")
      .def(
          "bytes_in_interval",
          [](ddl::NativeStager& st, uintptr_t e0, uintptr_t e1, int64_t timeout_ms) {
            ddl::InIntervalBytes r;
            {
              py::gil_scoped_release nogil;
              r = st.bytes_in_interval(reinterpret_cast<hipEvent_t>(e0), reinterpret_cast<hipEvent_t>(e1), timeout_ms);
            }
            py::dict d;
            d["ok"] = r.ok;
            d["bytes"] = r.bytes;
            d["windows"] = r.windows;
            d["copies"] = r.copies;
            d["t0_ms"] = r.t0_ms;
            d["t1_ms"] = r.t1_ms;
            d["busy_ms"] = r.busy_ms;
            d["overlap_ms"] = r.overlap_ms;
            d["copies_per_stream"] = py::make_tuple(r.copies_per_stream[0], r.copies_per_stream[1]);
            d["untimed"] = r.untimed;
            d["truncated"] = r.truncated;
            return d;
          },
          py::arg("e0"), py::arg("e1"), py::arg("timeout_ms") = 2000,
          "H2D bytes that crossed PCIe between two completed timing events (device clock, pro rata per copy)")
      .def_property_readonly("wait_log", &ddl::NativeStager::wait_log,
                             "per staged window (first 4096): [window, ns ring wait, ns free-event wait enqueue, "
                             "ns producer wait, ns copy enqueue, ns retire slot + event records, t0 ns]");

  // ------------------------------------------------- native batch dispatch
  py::class_<ddl::BatchEngine>(m, "BatchEngine")
      .def(py::init([](ddl::NativeStager& stager, int kind, int in_dt, int out_dt, bool shuffle, int64_t batch,
                       int64_t row_elems, uint64_t seed, std::vector<int64_t> n_data, std::vector<int32_t> widths,
                       std::vector<float> scale, std::vector<float> bias, int64_t plane, int64_t max_blocks,
                       int32_t n_producers, std::vector<uintptr_t> buffers, std::vector<uintptr_t> ready,
                       uintptr_t batch_stream, int device, std::vector<int64_t> token, std::vector<double> augment,
                       uint64_t aug_seed) {
             ddl::BatchRecipe r;
             r.kind = kind;
             r.in_dt = in_dt;
             r.out_dt = out_dt;
             r.shuffle = shuffle ? 1 : 0;
             r.batch = batch;
             r.row_elems = row_elems;
             r.seed = seed;
             r.max_blocks = max_blocks;
             r.n_data = std::move(n_data);
             r.widths = std::move(widths);
             r.aff = make_affine(scale, bias, plane);
             if (kind == 2) {
               if (token.size() != 10 && token.size() != 11)
                 throw std::invalid_argument("BatchEngine: token recipe needs 10 or 11 values");
               r.token_mode = static_cast<int32_t>(token[0]);
               r.pad_id = static_cast<int32_t>(token[1]);
               r.seq_len = token[2];
               r.off_offsets = token[3];
               r.off_row_start = token[4];
               r.off_row_end = token[5];
               r.off_seg_offsets = token[6];
               r.off_tokens = token[7];
               r.header_stride = token[8];
               r.token_fill_rows = token[9];
               r.token_bytes = token.size() > 10 ? token[10] : 4;
               if (r.token_bytes != 4 && r.token_bytes != 2)
                 throw std::invalid_argument("BatchEngine: tokens are 4 (int32) or 2 (uint16) bytes");
             }
             if (kind == 4) {
               if (augment.size() != 11)
                 throw std::invalid_argument("BatchEngine: augment recipe needs 11 values");
               r.aug_hwc = static_cast<int32_t>(augment[0]);
               r.aug.in_h = static_cast<int32_t>(augment[1]);
               r.aug.in_w = static_cast<int32_t>(augment[2]);
               r.aug.channels = static_cast<int32_t>(augment[3]);
               r.aug.out_h = static_cast<int32_t>(augment[4]);
               r.aug.out_w = static_cast<int32_t>(augment[5]);
               r.aug.scale_min = static_cast<float>(augment[6]);
               r.aug.scale_max = static_cast<float>(augment[7]);
               r.aug.ratio_min = static_cast<float>(augment[8]);
               r.aug.ratio_max = static_cast<float>(augment[9]);
               r.aug.flip_p = static_cast<float>(augment[10]);
               r.aug_seed = aug_seed;
             }
             std::vector<void*> bufs;
             for (auto b : buffers) bufs.push_back(as_ptr<void>(b));
             std::vector<hipEvent_t> rd;
             for (auto e : ready) rd.push_back(reinterpret_cast<hipEvent_t>(e));
             return std::make_unique<ddl::BatchEngine>(&stager, std::move(r), n_producers, std::move(bufs),
                                                       std::move(rd), as_stream(batch_stream), device);
           }),
           py::arg("stager"), py::arg("kind"), py::arg("in_dt"), py::arg("out_dt"), py::arg("shuffle"),
           py::arg("batch"), py::arg("row_elems"), py::arg("seed"), py::arg("n_data"), py::arg("widths"),
           py::arg("scale"), py::arg("bias"), py::arg("plane"), py::arg("max_blocks"), py::arg("n_producers"),
           py::arg("buffers"), py::arg("ready"), py::arg("batch_stream"), py::arg("device"),
           py::arg("token") = std::vector<int64_t>{}, py::arg("augment") = std::vector<double>{},
           py::arg("aug_seed") = 0, py::keep_alive<1, 2>(),
           "token = [mode (0 pad, 1 pack), pad_id, seq_len, byte offsets of offsets, row_start, row_end, "
           "seg_offsets, tokens] for kind 2")
      .def("set_epoch_base", &ddl::BatchEngine::set_epoch_base, py::arg("window0"), py::arg("epoch0"),
           py::arg("windows_per_epoch"),
           "augment (kind 4): window window0 starts epoch epoch0; the crop seed of window w mixes in its epoch")
      .def(
          "provide",
          [](ddl::BatchEngine& e, const std::vector<std::vector<uintptr_t>>& slots) {
            std::vector<std::vector<void*>> v;
            v.reserve(slots.size());
            for (const auto& s : slots) {
              std::vector<void*> o;
              for (auto p : s) o.push_back(as_ptr<void>(p));
              v.push_back(std::move(o));
            }
            e.provide(v);
          },
          py::arg("slots"))
      .def_property_readonly("slots_left", &ddl::BatchEngine::slots_left)
      .def(
          "get",
          [](ddl::BatchEngine& e, int64_t w, int64_t local, int64_t bpw, bool next_ok, uintptr_t compute,
             int64_t timeout_ms) {
            int32_t fp = -1;
            int64_t slot;
            int64_t tags[4] = {0, 0, 0, 0};
            {
              py::gil_scoped_release nogil;
              slot = e.get(w, local, bpw, next_ok, as_stream(compute), timeout_ms, &fp, tags);
            }
            return py::make_tuple(slot, slot >= 0 ? int32_t{-1} : fp, py::make_tuple(tags[0], tags[1], tags[2], tags[3]));
          },
          py::arg("window"), py::arg("local"), py::arg("bpw"), py::arg("next_ok"), py::arg("compute_stream"),
          py::arg("timeout_ms"),
          "(slot, -1, window tags) for batch `local` of window `window`, else (code, producer, _): "
          "-(10 + stager wait code) if the window could not be staged, -1 HIP error, -2 no output slot")
      .def(
          "acquire",
          [](ddl::BatchEngine& e, int64_t w, int64_t timeout_ms) {
            int32_t fp = -1;
            int rc;
            {
              py::gil_scoped_release nogil;
              rc = e.acquire(w, timeout_ms, &fp);
            }
            return py::make_tuple(rc, fp);
          },
          py::arg("window"), py::arg("timeout_ms"))
      .def("release", &ddl::BatchEngine::release, py::arg("window"), py::call_guard<py::gil_scoped_release>(),
           "hand window w back to the stager (0 ok; -4: the bounded wait for its copy failed, -1 HIP error)")
      .def("reset", &ddl::BatchEngine::reset)
      .def_property("inline", &ddl::BatchEngine::is_inline, &ddl::BatchEngine::set_inline)
      .def("set_window_mode", &ddl::BatchEngine::set_window_mode, py::arg("on"), py::arg("slot_stride"))
      .def_property_readonly("window_mode", &ddl::BatchEngine::window_mode)
      .def_property("early_release", &ddl::BatchEngine::early_release, &ddl::BatchEngine::set_early_release)
      .def("set_batches_per_window", &ddl::BatchEngine::set_batches_per_window, py::arg("bpw"))
      .def_property("host_handoff", &ddl::BatchEngine::host_handoff, &ddl::BatchEngine::set_host_handoff)
      .def_property("ready_on_host", &ddl::BatchEngine::ready_on_host, &ddl::BatchEngine::set_ready_on_host)
      .def_property("ready_event_on_host", &ddl::BatchEngine::ready_event_on_host,
                    &ddl::BatchEngine::set_ready_event_on_host)
      .def_property_readonly("ready_host_waits", &ddl::BatchEngine::ready_host_waits)
      .def_property_readonly("wait_s", &ddl::BatchEngine::wait_s)
      .def_property_readonly("batches", &ddl::BatchEngine::batches)
      .def_property_readonly("lookahead_hits", &ddl::BatchEngine::lookahead_hits)
      .def_property_readonly("timing_ns", &ddl::BatchEngine::timing_ns)
      .def_property_readonly("compute_waits", &ddl::BatchEngine::compute_waits);
  m.def(
      "host_feistel_keys",
      [](uint64_t seed, uint64_t key, uint64_t n) {
        const ddl::FeistelKeys k = ddl::host_feistel_keys(seed, key, n);
        std::vector<uint64_t> keys(k.k, k.k + ddl::kFeistelRounds);
        return py::make_tuple(keys, k.half_bits);
      },
      py::arg("seed"), py::arg("key"), py::arg("n"), "Feistel round keys + half bits of (seed, key) over [0, n)");
  m.def("host_window_perm_key", &ddl::host_window_perm_key, py::arg("producer"), py::arg("round"));
  m.def(
      "bucket_send",
      [](std::vector<uint64_t> keys, uint64_t n_domain, uint32_t half_bits, int64_t pos0, int64_t count,
         int64_t shard_rows, int64_t lo, int32_t rank, int32_t world, uintptr_t out, uintptr_t stream) {
        ddl::BucketSpec sp{};
        sp.keys = make_keys(keys, n_domain, half_bits);
        sp.pos0 = pos0;
        sp.count = count;
        sp.shard_rows = shard_rows;
        sp.lo = lo;
        sp.rank = rank;
        sp.world = world;
        check_rc(ddl::bucket_send(sp, as_ptr<int64_t>(out), as_stream(stream)), "bucket_send");
      },
      py::arg("keys"), py::arg("n_domain"), py::arg("half_bits"), py::arg("pos0"), py::arg("count"),
      py::arg("shard_rows"), py::arg("lo"), py::arg("rank"), py::arg("world"), py::arg("out"), py::arg("stream"));
  m.def(
      "bucket_recv",
      [](std::vector<uint64_t> keys, uint64_t n_domain, uint32_t half_bits, int64_t pos0, int64_t count,
         int64_t shard_rows, int32_t world, std::vector<int64_t> offsets, uintptr_t out, uintptr_t stream) {
        if (offsets.size() != static_cast<size_t>(world) || world > ddl::kMaxBucketWorld)
          throw std::invalid_argument("bucket_recv: one offset per rank, world <= 64");
        ddl::BucketSpec sp{};
        sp.keys = make_keys(keys, n_domain, half_bits);
        sp.pos0 = pos0;
        sp.count = count;
        sp.shard_rows = shard_rows;
        sp.world = world;
        for (int q = 0; q < world; ++q) sp.offsets[q] = offsets[q];
        check_rc(ddl::bucket_recv(sp, as_ptr<int64_t>(out), as_stream(stream)), "bucket_recv");
      },
      py::arg("keys"), py::arg("n_domain"), py::arg("half_bits"), py::arg("pos0"), py::arg("count"),
      py::arg("shard_rows"), py::arg("world"), py::arg("offsets"), py::arg("out"), py::arg("stream"));

  m.def(
      "api_costs",
      [](int iters) {
        // host cost (us per call) of the HIP calls on the per-batch path, on two fresh streams
        hipStream_t a, b;
        hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
        hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
        hipEvent_t ev;
        hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        void* flag = nullptr;
        hipMalloc(&flag, 64);
        hipMemsetAsync(flag, 0, 64, a);
        hipStreamSynchronize(a);
        auto t = [&](auto fn) {
          for (int i = 0; i < 50; ++i) fn(i);
          hipDeviceSynchronize();
          const auto t0 = std::chrono::steady_clock::now();
          for (int i = 0; i < iters; ++i) fn(i);
          const double us =
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
          hipDeviceSynchronize();
          return us;
        };
        py::dict d;
        d["hipEventRecord"] = t([&](int) { hipEventRecord(ev, a); });
        d["hipStreamWaitEvent"] = t([&](int) { hipStreamWaitEvent(b, ev, 0); });
        d["hipEventQuery"] = t([&](int) { (void)hipEventQuery(ev); });
        d["record+wait"] = t([&](int) {
          hipEventRecord(ev, a);
          hipStreamWaitEvent(b, ev, 0);
        });
        d["hipStreamWriteValue64"] = t([&](int i) { hipStreamWriteValue64(a, flag, static_cast<uint64_t>(i), 0); });
        d["hipStreamWaitValue64"] = t([&](int i) {
          hipStreamWaitValue64(b, flag, 0, hipStreamWaitValueGte, 0xFFFFFFFFFFFFFFFFull);
        });
        d["hipMemsetAsync 4B"] = t([&](int) { hipMemsetAsync(flag, 0, 4, a); });
        hipDeviceSynchronize();
        hipFree(flag);
        hipEventDestroy(ev);
        hipStreamDestroy(a);
        hipStreamDestroy(b);
        return d;
      },
      py::arg("iters") = 20000, "Host microseconds per call of the HIP stream/event APIs on the batch path");

  // --------------------------------------------------------------- kernels
  m.def(
      "gather_rows",
      [](uintptr_t dst, int out_dt, uintptr_t src, int in_dt, int64_t n_rows, int64_t row_elems, int mode,
         uintptr_t idx, int64_t base, std::vector<uint64_t> keys, uint64_t n_domain, uint32_t half_bits,
         std::vector<float> scale, std::vector<float> bias, int64_t plane, bool scatter, uintptr_t stream,
         int64_t max_blocks, bool host_src) {
        const ddl::RowIndex ri = make_index(mode, idx, base, keys, n_domain, half_bits);
        const ddl::Affine aff = make_affine(scale, bias, plane);
        check_rc(ddl::gather_rows(as_ptr<void>(dst), out_dt, as_ptr<const void>(src), in_dt, n_rows, row_elems, ri,
                                  aff, (scatter ? 1 : 0) | (host_src ? ddl::kHostSource : 0), max_blocks,
                                  as_stream(stream)),
                 "gather_rows");
      },
      py::arg("dst"), py::arg("out_dt"), py::arg("src"), py::arg("in_dt"), py::arg("n_rows"), py::arg("row_elems"),
      py::arg("mode"), py::arg("idx"), py::arg("base"), py::arg("keys"), py::arg("n_domain"), py::arg("half_bits"),
      py::arg("scale"), py::arg("bias"), py::arg("plane"), py::arg("scatter"), py::arg("stream"),
      py::arg("max_blocks") = 0, py::arg("host_src") = false);
  m.def(
      "feistel_indices",
      [](uintptr_t out, int64_t count, int64_t base, std::vector<uint64_t> keys, uint64_t n_domain,
         uint32_t half_bits, uintptr_t stream) {
        check_rc(ddl::feistel_indices(as_ptr<int64_t>(out), count, base, make_keys(keys, n_domain, half_bits),
                                      as_stream(stream)),
                 "feistel_indices");
      },
      py::arg("out"), py::arg("count"), py::arg("base"), py::arg("keys"), py::arg("n_domain"), py::arg("half_bits"),
      py::arg("stream"));
  m.def(
      "collate_hwc_to_chw",
      [](uintptr_t dst, int out_dt, uintptr_t src, int in_dt, int64_t batch, int64_t pixels, int channels, int mode,
         uintptr_t idx, int64_t base, std::vector<uint64_t> keys, uint64_t n_domain, uint32_t half_bits,
         std::vector<float> scale, std::vector<float> bias, uintptr_t stream) {
        const ddl::RowIndex ri = make_index(mode, idx, base, keys, n_domain, half_bits);
        const ddl::Affine aff = make_affine(scale, bias, pixels);
        check_rc(ddl::collate_hwc_to_chw(as_ptr<void>(dst), out_dt, as_ptr<const void>(src), in_dt, batch, pixels,
                                         channels, ri, aff, as_stream(stream)),
                 "collate_hwc_to_chw");
      },
      py::arg("dst"), py::arg("out_dt"), py::arg("src"), py::arg("in_dt"), py::arg("batch"), py::arg("pixels"),
      py::arg("channels"), py::arg("mode"), py::arg("idx"), py::arg("base"), py::arg("keys"), py::arg("n_domain"),
      py::arg("half_bits"), py::arg("scale"), py::arg("bias"), py::arg("stream"));
  m.def(
      "split_columns",
      [](std::vector<uintptr_t> dsts, std::vector<int> widths, int out_dt, uintptr_t src, int in_dt, int64_t n_rows,
         int64_t n_values, int mode, uintptr_t idx, int64_t base, std::vector<uint64_t> keys, uint64_t n_domain,
         uint32_t half_bits, uintptr_t stream) {
        if (dsts.size() != widths.size() || dsts.empty() || dsts.size() > 8)
          throw std::invalid_argument("split_columns: 1..8 groups");
        ddl::SplitSpec sp{};
        int64_t tot = 0;
        for (size_t i = 0; i < dsts.size(); ++i) {
          sp.dst[i] = as_ptr<void>(dsts[i]);
          sp.width[i] = widths[i];
          tot += widths[i];
        }
        if (tot != n_values) throw std::invalid_argument("split_columns: widths must sum to n_values");
        sp.n_groups = static_cast<int32_t>(dsts.size());
        sp.out_dt = out_dt;
        const ddl::RowIndex ri = make_index(mode, idx, base, keys, n_domain, half_bits);
        check_rc(ddl::split_columns(sp, as_ptr<const void>(src), in_dt, n_rows, n_values, ri, as_stream(stream)),
                 "split_columns");
      },
      py::arg("dsts"), py::arg("widths"), py::arg("out_dt"), py::arg("src"), py::arg("in_dt"), py::arg("n_rows"),
      py::arg("n_values"), py::arg("mode"), py::arg("idx"), py::arg("base"), py::arg("keys"), py::arg("n_domain"),
      py::arg("half_bits"), py::arg("stream"));
  m.def(
      "random_resized_crop",
      [](uintptr_t dst, int out_dt, uintptr_t src, int in_dt, int64_t batch, bool hwc, int in_h, int in_w, int channels,
         int out_h, int out_w, uint64_t seed, int64_t sample_base, float scale_min, float scale_max, float ratio_min,
         float ratio_max, float flip_p, int mode, uintptr_t idx, int64_t base, std::vector<uint64_t> keys,
         uint64_t n_domain, uint32_t half_bits, std::vector<float> scale, std::vector<float> bias, uintptr_t boxes_out,
         int path, uintptr_t stream, uintptr_t sample_ids) {
        ddl::AugmentSpec a{};
        a.seed = seed;
        a.sample_base = sample_base;
        a.sample_ids = as_ptr<const int64_t>(sample_ids);
        a.in_h = in_h;
        a.in_w = in_w;
        a.out_h = out_h;
        a.out_w = out_w;
        a.channels = channels;
        a.scale_min = scale_min;
        a.scale_max = scale_max;
        a.ratio_min = ratio_min;
        a.ratio_max = ratio_max;
        a.flip_p = flip_p;
        const ddl::RowIndex ri = make_index(mode, idx, base, keys, n_domain, half_bits);
        const ddl::Affine aff = make_affine(scale, bias, 1);
        check_rc(ddl::random_resized_crop(as_ptr<void>(dst), out_dt, as_ptr<const void>(src), in_dt, batch, a,
                                          hwc ? 1 : 0, ri, aff, as_ptr<int32_t>(boxes_out), path, as_stream(stream)),
                 "random_resized_crop");
      },
      py::arg("dst"), py::arg("out_dt"), py::arg("src"), py::arg("in_dt"), py::arg("batch"), py::arg("hwc"),
      py::arg("in_h"), py::arg("in_w"), py::arg("channels"), py::arg("out_h"), py::arg("out_w"), py::arg("seed"),
      py::arg("sample_base"), py::arg("scale_min"), py::arg("scale_max"), py::arg("ratio_min"), py::arg("ratio_max"),
      py::arg("flip_p"), py::arg("mode"), py::arg("idx"), py::arg("base"), py::arg("keys"), py::arg("n_domain"),
      py::arg("half_bits"), py::arg("scale"), py::arg("bias"), py::arg("boxes_out"), py::arg("path"),
      py::arg("stream"), py::arg("sample_ids") = 0);
  m.def(
      "pack_columns",
      [](std::vector<uintptr_t> srcs, std::vector<int> widths, int in_dt, uintptr_t dst, int out_dt, int64_t n_rows,
         int64_t n_values, int mode, uintptr_t idx, int64_t base, std::vector<uint64_t> keys, uint64_t n_domain,
         uint32_t half_bits, uintptr_t stream) {
        if (srcs.size() != widths.size() || srcs.empty() || srcs.size() > 8)
          throw std::invalid_argument("pack_columns: 1..8 groups");
        ddl::SplitSpec sp{};
        int64_t tot = 0;
        for (size_t i = 0; i < srcs.size(); ++i) {
          sp.dst[i] = as_ptr<void>(srcs[i]);
          sp.width[i] = widths[i];
          tot += widths[i];
        }
        if (tot != n_values) throw std::invalid_argument("pack_columns: widths must sum to n_values");
        sp.n_groups = static_cast<int32_t>(srcs.size());
        sp.out_dt = out_dt;
        const ddl::RowIndex ri = make_index(mode, idx, base, keys, n_domain, half_bits);
        check_rc(ddl::pack_columns(sp, as_ptr<void>(dst), in_dt, n_rows, n_values, ri, as_stream(stream)),
                 "pack_columns");
      },
      py::arg("srcs"), py::arg("widths"), py::arg("in_dt"), py::arg("dst"), py::arg("out_dt"), py::arg("n_rows"),
      py::arg("n_values"), py::arg("mode"), py::arg("idx"), py::arg("base"), py::arg("keys"), py::arg("n_domain"),
      py::arg("half_bits"), py::arg("stream"));
  m.def(
      "pad_pack_tokens",
      [](uintptr_t tokens, uintptr_t offsets, uintptr_t row_start, uintptr_t row_end, uintptr_t seg_offsets,
         int64_t n_seg, uintptr_t out_tokens, uintptr_t attn_mask, uintptr_t position_ids, bool pos_is_i64,
         uintptr_t segment_ids, uintptr_t cu_seqlens_out, int64_t rows, int64_t seq_len, int pad_id, int mode,
         uintptr_t stream, int64_t fill_rows, uintptr_t dev_counts, bool tok16) {
        ddl::TokenSpec sp{};
        sp.tok16 = tok16 ? 1 : 0;
        sp.fill_rows = fill_rows;
        sp.dev_counts = as_ptr<const int64_t>(dev_counts);
        sp.tokens = as_ptr<const void>(tokens);
        sp.offsets = as_ptr<const int64_t>(offsets);
        sp.row_start = as_ptr<const int64_t>(row_start);
        sp.row_end = as_ptr<const int64_t>(row_end);
        sp.seg_offsets = as_ptr<const int64_t>(seg_offsets);
        sp.n_seg = n_seg;
        sp.out_tokens = as_ptr<int32_t>(out_tokens);
        sp.attn_mask = as_ptr<uint8_t>(attn_mask);
        sp.position_ids = as_ptr<void>(position_ids);
        sp.pos_is_i64 = pos_is_i64 ? 1 : 0;
        sp.segment_ids = as_ptr<int32_t>(segment_ids);
        sp.cu_seqlens_out = as_ptr<int32_t>(cu_seqlens_out);
        sp.rows = rows;
        sp.seq_len = seq_len;
        sp.pad_id = pad_id;
        sp.mode = mode;
        check_rc(ddl::pad_pack_tokens(sp, as_stream(stream)), "pad_pack_tokens");
      },
      py::arg("tokens"), py::arg("offsets"), py::arg("row_start"), py::arg("row_end"), py::arg("seg_offsets"),
      py::arg("n_seg"), py::arg("out_tokens"), py::arg("attn_mask"), py::arg("position_ids"), py::arg("pos_is_i64"),
      py::arg("segment_ids"), py::arg("cu_seqlens_out"), py::arg("rows"), py::arg("seq_len"), py::arg("pad_id"),
      py::arg("mode"), py::arg("stream"), py::arg("fill_rows") = 0, py::arg("dev_counts") = 0,
      py::arg("tok16") = false);
  m.def("pack_plan_scratch_ints", &ddl::pack_plan_scratch_ints, py::arg("max_segs"), py::arg("max_rows"));
  m.def(
      "pack_plan_device",
      [](uintptr_t offsets, int64_t n, int64_t seq_len, int64_t max_segs, int64_t max_rows, uintptr_t seg_offsets,
         uintptr_t row_start, uintptr_t row_end, uintptr_t counts, uintptr_t scratch, uintptr_t stream) {
        ddl::PackPlanSpec sp{};
        sp.offsets = as_ptr<const int64_t>(offsets);
        sp.n = n;
        sp.seq_len = seq_len;
        sp.max_segs = max_segs;
        sp.max_rows = max_rows;
        sp.seg_offsets = as_ptr<int64_t>(seg_offsets);
        sp.row_start = as_ptr<int64_t>(row_start);
        sp.row_end = as_ptr<int64_t>(row_end);
        sp.counts = as_ptr<int64_t>(counts);
        sp.scratch = as_ptr<int32_t>(scratch);
        check_rc(ddl::pack_plan_device(sp, as_stream(stream)), "pack_plan_device");
      },
      py::arg("offsets"), py::arg("n"), py::arg("seq_len"), py::arg("max_segs"), py::arg("max_rows"),
      py::arg("seg_offsets"), py::arg("row_start"), py::arg("row_end"), py::arg("counts"), py::arg("scratch"),
      py::arg("stream"));
  m.def(
      "touch_pages",
      [](uintptr_t ptr, int64_t bytes, int64_t page, uintptr_t sink, int blocks, uintptr_t stream) {
        check_rc(ddl::touch_pages(as_ptr<const void>(ptr), bytes, page, as_ptr<uint32_t>(sink), blocks,
                                  as_stream(stream)),
                 "touch_pages");
      },
      py::arg("ptr"), py::arg("bytes"), py::arg("page"), py::arg("sink"), py::arg("blocks"), py::arg("stream"));
  m.def(
      "stream_copy",
      [](uintptr_t src, uintptr_t dst, int64_t bytes, int blocks, uintptr_t stream) {
        check_rc(ddl::stream_copy(as_ptr<const void>(src), as_ptr<void>(dst), bytes, blocks,
                                  reinterpret_cast<hipStream_t>(stream)),
                 "stream_copy");
      },
      py::arg("src"), py::arg("dst"), py::arg("bytes"), py::arg("blocks"), py::arg("stream"));
  m.def(
      "checksum_words",
      [](uintptr_t ptr, int64_t bytes, uintptr_t out, uintptr_t scratch, int64_t scratch_len, uintptr_t stream) {
        check_rc(ddl::checksum_words(as_ptr<const void>(ptr), bytes, as_ptr<uint64_t>(out), as_ptr<uint64_t>(scratch),
                                     scratch_len, as_stream(stream)),
                 "checksum_words");
      },
      py::arg("ptr"), py::arg("bytes"), py::arg("out"), py::arg("scratch"), py::arg("scratch_len"),
      py::arg("stream"));
  m.attr("CHECKSUM_MAX_BLOCKS") = ddl::kChecksumMaxBlocks;
  m.def(
      "checksum_accumulate",
      [](uintptr_t ptr, int64_t bytes, uintptr_t partials, int64_t n_partials, uintptr_t stream) {
        check_rc(ddl::checksum_accumulate(as_ptr<const void>(ptr), bytes, as_ptr<uint64_t>(partials), n_partials,
                                          as_stream(stream)),
                 "checksum_accumulate");
      },
      py::arg("ptr"), py::arg("bytes"), py::arg("partials"), py::arg("n_partials"), py::arg("stream"));
  m.def(
      "checksum_finalize",
      [](uintptr_t partials, int64_t n_partials, uintptr_t out, uintptr_t stream) {
        check_rc(ddl::checksum_finalize(as_ptr<const uint64_t>(partials), n_partials, as_ptr<uint64_t>(out),
                                        as_stream(stream)),
                 "checksum_finalize");
      },
      py::arg("partials"), py::arg("n_partials"), py::arg("out"), py::arg("stream"));
  m.def(
      "column_stats",
      [](uintptr_t src, int64_t n, int64_t cols, uintptr_t sum, uintptr_t sumsq, uintptr_t mn, uintptr_t mx,
         uintptr_t stream) {
        check_rc(ddl::column_stats(as_ptr<const float>(src), n, cols, as_ptr<float>(sum), as_ptr<float>(sumsq),
                                   as_ptr<float>(mn), as_ptr<float>(mx), as_stream(stream)),
                 "column_stats");
      },
      py::arg("src"), py::arg("n"), py::arg("cols"), py::arg("sum"), py::arg("sumsq"), py::arg("min"), py::arg("max"),
      py::arg("stream"));
}
