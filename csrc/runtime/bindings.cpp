// pybind11 bindings for the host runtime: module ddl_amd._ddl_runtime.
// No torch / HIP dependency: this module works on CPU-only hosts (the
// producer worker processes never touch the GPU).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>
#include <new>

#include "arena.h"
#include "feistel.h"
#include <algorithm>
#include "fileio.h"
#include "numa.h"

namespace py = pybind11;
using ddl::Arena;

namespace {

py::dict slot_info(const Arena& a, uint32_t p, uint32_t s) {
  ddl::SlotHeader* sh = a.slot(p, s);
  py::dict d;
  d["state"] = sh->state.load();
  d["offset"] = sh->offset;
  d["capacity"] = sh->capacity;
  d["seq"] = sh->seq.load();
  d["used_bytes"] = sh->used_bytes.load();
  d["epoch"] = sh->epoch.load();
  d["publish_ns"] = sh->publish_ns.load();
  py::list tags;
  for (auto& t : sh->tag) tags.append(t.load());
  d["tag"] = tags;
  return d;
}

}  // namespace

PYBIND11_MODULE(_ddl_runtime, m) {
  m.doc() = "ddl_amd native host runtime: shm slot arena, futex hand-off, host gather";

  py::enum_<ddl::WaitResult>(m, "WaitResult")
      .value("OK", ddl::kOk)
      .value("SHUTDOWN", ddl::kShutdown)
      .value("TIMEOUT", ddl::kTimeout)
      .value("PEER_DEAD", ddl::kPeerDead)
      .value("PEER_FAILED", ddl::kPeerFailed);

  m.attr("EMPTY") = static_cast<uint32_t>(ddl::kEmpty);
  m.attr("READY") = static_cast<uint32_t>(ddl::kReady);
  m.attr("HELD") = static_cast<uint32_t>(ddl::kHeld);
  m.attr("STATUS_INIT") = static_cast<uint32_t>(ddl::kStatusInit);
  m.attr("STATUS_RUNNING") = static_cast<uint32_t>(ddl::kStatusRunning);
  m.attr("STATUS_DONE") = static_cast<uint32_t>(ddl::kStatusDone);
  m.attr("STATUS_FAILED") = static_cast<uint32_t>(ddl::kStatusFailed);
  m.attr("DATA_ALIGN") = ddl::kDataAlign;
  m.attr("ARENA_ABI") = ddl::arena_abi();

  m.def("now_ns", &ddl::now_ns);
  m.def("pid_alive", &ddl::pid_alive, py::arg("pid"));

  py::class_<Arena, std::unique_ptr<Arena>>(m, "Arena")
      .def_static(
          "create",
          [](const std::string& name, const std::vector<uint64_t>& caps, uint32_t n_slots) {
            return std::unique_ptr<Arena>(Arena::create(name, caps, n_slots));
          },
          py::arg("name"), py::arg("capacities"), py::arg("n_slots"))
      .def_static(
          "attach", [](const std::string& name) { return std::unique_ptr<Arena>(Arena::attach(name)); },
          py::arg("name"))
      .def("unlink", &Arena::unlink)
      .def_property_readonly("name", &Arena::name)
      .def_property_readonly("address", [](const Arena& a) { return reinterpret_cast<uintptr_t>(&a); },
                             "address of this C++ Arena object (for the HIP extension's native stager)")
      .def_property_readonly("base_address",
                             [](const Arena& a) { return reinterpret_cast<uintptr_t>(a.base()); })
      .def_property_readonly("total_bytes", &Arena::total_bytes)
      .def_property_readonly("data_offset", &Arena::data_offset)
      .def_property_readonly("n_producers", &Arena::n_producers)
      .def_property_readonly("n_slots", &Arena::n_slots)
      .def("slot_address",
           [](const Arena& a, uint32_t p, uint32_t s) {
             return reinterpret_cast<uintptr_t>(a.slot_data(p, s));
           })
      .def("state_address",
           [](const Arena& a, uint32_t p, uint32_t s) {
             return reinterpret_cast<uintptr_t>(&a.slot(p, s)->state);
           })
      .def("slot_capacity", [](const Arena& a, uint32_t p, uint32_t s) { return a.slot(p, s)->capacity; })
      .def(
          "slot_view",
          [](const Arena& a, uint32_t p, uint32_t s) {
            ddl::SlotHeader* sh = a.slot(p, s);
            return py::memoryview::from_memory(a.base() + sh->offset,
                                               static_cast<py::ssize_t>(sh->capacity), false);
          },
          py::arg("producer"), py::arg("slot"))
      .def("slot_info", [](const Arena& a, uint32_t p, uint32_t s) { return slot_info(a, p, s); })
      .def(
          "wait_state",
          [](const Arena& a, uint32_t p, uint32_t s, uint32_t expected, int64_t timeout_ms,
             int32_t peer_pid, int32_t producer_index) {
            py::gil_scoped_release nogil;
            return a.wait_state(p, s, expected, timeout_ms, peer_pid, producer_index);
          },
          py::arg("producer"), py::arg("slot"), py::arg("expected"), py::arg("timeout_ms") = -1,
          py::arg("peer_pid") = 0, py::arg("producer_index") = -1)
      .def("set_state", &Arena::set_state)
      .def("cas_state", &Arena::cas_state)
      .def("get_state", &Arena::get_state)
      .def(
          "publish",
          [](const Arena& a, uint32_t p, uint32_t s, uint64_t seq, uint64_t used, uint64_t epoch,
             std::vector<int64_t> tags) {
            ddl::SlotHeader* sh = a.slot(p, s);
            if (used > sh->capacity) throw std::out_of_range("publish: used_bytes > capacity");
            sh->seq.store(seq, std::memory_order_relaxed);
            sh->used_bytes.store(used, std::memory_order_relaxed);
            sh->epoch.store(epoch, std::memory_order_relaxed);
            for (size_t i = 0; i < tags.size() && i < 4; ++i)
              sh->tag[i].store(tags[i], std::memory_order_relaxed);
            sh->publish_ns.store(ddl::now_ns(), std::memory_order_relaxed);
            a.set_state(p, s, ddl::kReady);  // release: orders every store above
          },
          py::arg("producer"), py::arg("slot"), py::arg("seq"), py::arg("used_bytes"),
          py::arg("epoch") = 0, py::arg("tags") = std::vector<int64_t>{})
      .def("request_shutdown", &Arena::request_shutdown)
      .def("shutdown_requested", &Arena::shutdown_requested)
      .def("mark_failed", &Arena::mark_failed)
      .def("failed_producer", &Arena::failed_producer)
      .def("attached", [](const Arena& a) { return a.header()->attached.load(); })
      .def("set_producer_pid",
           [](const Arena& a, uint32_t p, int32_t pid) {
             a.producer(p)->pid.store(pid);
             a.producer(p)->status.store(ddl::kStatusRunning, std::memory_order_release);
           })
      .def("set_producer_status",
           [](const Arena& a, uint32_t p, uint32_t st) {
             a.producer(p)->status.store(st, std::memory_order_release);
           })
      .def("heartbeat",
           [](const Arena& a, uint32_t p, uint64_t fill_ns, uint64_t wait_ns) {
             ddl::ProducerRecord* r = a.producer(p);
             r->heartbeat_ns.store(ddl::now_ns(), std::memory_order_relaxed);
             r->rounds.fetch_add(1, std::memory_order_relaxed);
             r->fill_ns_total.fetch_add(fill_ns, std::memory_order_relaxed);
             r->wait_ns_total.fetch_add(wait_ns, std::memory_order_relaxed);
           })
      .def("producer_info", [](const Arena& a, uint32_t p) {
        ddl::ProducerRecord* r = a.producer(p);
        py::dict d;
        d["pid"] = r->pid.load();
        d["status"] = r->status.load();
        d["heartbeat_ns"] = r->heartbeat_ns.load();
        d["rounds"] = r->rounds.load();
        d["fill_ns_total"] = r->fill_ns_total.load();
        d["wait_ns_total"] = r->wait_ns_total.load();
        return d;
      });

  m.def(
      "gather_rows",
      [](uintptr_t dst, uintptr_t src, uint64_t row_bytes, py::array_t<int64_t, py::array::c_style> idx,
         uint64_t src_rows, int n_threads) {
        const int64_t* ip = idx.data();
        const uint64_t n = static_cast<uint64_t>(idx.size());
        py::gil_scoped_release nogil;
        ddl::gather_rows(reinterpret_cast<uint8_t*>(dst), reinterpret_cast<const uint8_t*>(src),
                         row_bytes, ip, n, src_rows, n_threads);
      },
      py::arg("dst"), py::arg("src"), py::arg("row_bytes"), py::arg("indices"), py::arg("src_rows"),
      py::arg("n_threads") = 4,
      "dst[i*row_bytes:(i+1)*row_bytes] = src[idx[i]*row_bytes:...] on a host worker pool");
  m.def(
      "copy_spans",
      [](py::array_t<uint64_t, py::array::c_style> dst, py::array_t<uint64_t, py::array::c_style> src,
         py::array_t<uint64_t, py::array::c_style> sizes, int n_threads) {
        const py::ssize_t n = sizes.size();
        if (dst.size() != n || src.size() != n) throw std::invalid_argument("copy_spans: length mismatch");
        const auto* d = reinterpret_cast<const uintptr_t*>(dst.data());
        const auto* s = reinterpret_cast<const uintptr_t*>(src.data());
        const uint64_t* z = sizes.data();
        py::gil_scoped_release nogil;
        ddl::copy_spans(d, s, z, static_cast<uint64_t>(n), n_threads);
      },
      py::arg("dst"), py::arg("src"), py::arg("sizes"), py::arg("n_threads") = 4,
      "memcpy(dst[i], src[i], sizes[i]) for every i on the host worker pool, without the GIL");
  m.def(
      "feistel",
      [](std::vector<uint64_t> keys, uint32_t half_bits, uint64_t n, py::array_t<int64_t, py::array::c_style> pos) {
        if (keys.size() != ddl::kHostFeistelRounds) throw std::invalid_argument("feistel: need 6 round keys");
        auto out = py::array_t<int64_t>(pos.request().shape);
        const int64_t* in = pos.data();
        int64_t* o = out.mutable_data();
        const py::ssize_t m = pos.size();
        for (py::ssize_t i = 0; i < m; ++i) {
          if (in[i] < 0 || static_cast<uint64_t>(in[i]) >= n) throw std::out_of_range("feistel: position out of range");
        }
        {
          py::gil_scoped_release nogil;
          for (py::ssize_t i = 0; i < m; ++i)
            o[i] = static_cast<int64_t>(ddl::host_feistel_perm(static_cast<uint64_t>(in[i]), keys.data(), half_bits, n));
        }
        return out;
      },
      py::arg("keys"), py::arg("half_bits"), py::arg("n"), py::arg("positions"),
      "perm(positions) of the 6-round Feistel permutation (bit-identical to the gfx950 kernels)");
  m.def(
      "in_order_rows",
      [](py::array_t<int64_t, py::array::c_style> lengths, int64_t seq_len) {
        if (seq_len < 1) throw std::invalid_argument("in_order_rows: seq_len must be >= 1");
        const int64_t* l = lengths.data();
        const py::ssize_t m = lengths.size();
        int64_t rows = 0, cur = seq_len;  // cur = tokens in the open row (seq_len: no open row)
        for (py::ssize_t i = 0; i < m; ++i) {
          for (int64_t n = l[i]; n > 0;) {
            const int64_t seg = n < seq_len ? n : seq_len;
            if (cur + seg > seq_len) {
              ++rows;
              cur = 0;
            }
            cur += seg;
            n -= seg;
          }
        }
        return rows;
      },
      py::arg("lengths"), py::arg("seq_len"),
      "rows that in-order packing (pack_plan) of sequences of these lengths produces");
  m.def(
      "owner_counts",
      [](std::vector<uint64_t> keys, uint32_t half_bits, uint64_t n, int64_t pos0, int64_t gb, int64_t lb,
         int64_t shard_rows, int64_t world, int64_t rank) {
        if (keys.size() != ddl::kHostFeistelRounds) throw std::invalid_argument("owner_counts: need 6 round keys");
        if (lb <= 0 || shard_rows <= 0 || world < 1 || rank < 0 || rank >= world || pos0 < 0 ||
            static_cast<uint64_t>(pos0 + gb) > n)
          throw std::invalid_argument("owner_counts: bad geometry");
        std::vector<int64_t> send(world, 0), recv(world, 0);
        {
          py::gil_scoped_release nogil;
          for (int64_t i = 0; i < gb; ++i) {
            const int64_t idx = static_cast<int64_t>(
                ddl::host_feistel_perm(static_cast<uint64_t>(pos0 + i), keys.data(), half_bits, n));
            const int64_t owner = idx / shard_rows, dest = i / lb;
            if (owner == rank) ++send[dest];
            if (dest == rank) ++recv[owner];
          }
        }
        return py::make_tuple(send, recv);
      },
      py::arg("keys"), py::arg("half_bits"), py::arg("n"), py::arg("pos0"), py::arg("gb"), py::arg("lb"),
      py::arg("shard_rows"), py::arg("world"), py::arg("rank"),
      "(send_counts, recv_counts) of one global batch: samples this rank sends to / receives from every rank "
      "(sample idx lives on rank idx / shard_rows, position i goes to rank i / lb)");
  m.def(
      "owner_maps",
      [](std::vector<uint64_t> keys, uint32_t half_bits, uint64_t n, int64_t pos0, int64_t gb, int64_t lb,
         int64_t shard_rows, int64_t world, int64_t rank, int64_t lo) {
        // host twin of bucket.hip (CPU rehearsals): send list (own samples in position order, shard-local)
        // and receive map (row of each local position in the all-to-all receive buffer)
        if (keys.size() != ddl::kHostFeistelRounds) throw std::invalid_argument("owner_maps: need 6 round keys");
        if (lb <= 0 || shard_rows <= 0 || world < 1 || rank < 0 || rank >= world || pos0 < 0 ||
            static_cast<uint64_t>(pos0 + gb) > n)
          throw std::invalid_argument("owner_maps: bad geometry");
        std::vector<int64_t> owner(gb), send;
        std::vector<int64_t> recv_counts(world, 0);
        auto inv = py::array_t<int64_t>(lb);
        int64_t* iv = inv.mutable_data();
        {
          py::gil_scoped_release nogil;
          for (int64_t i = 0; i < gb; ++i) {
            const int64_t idx = static_cast<int64_t>(
                ddl::host_feistel_perm(static_cast<uint64_t>(pos0 + i), keys.data(), half_bits, n));
            owner[i] = idx / shard_rows;
            if (owner[i] == rank) send.push_back(idx - lo);
          }
          for (int64_t j = 0; j < lb; ++j) ++recv_counts[owner[rank * lb + j]];
          std::vector<int64_t> next(world, 0);
          for (int64_t q = 1; q < world; ++q) next[q] = next[q - 1] + recv_counts[q - 1];
          for (int64_t j = 0; j < lb; ++j) iv[j] = next[owner[rank * lb + j]]++;
        }
        auto sa = py::array_t<int64_t>(static_cast<py::ssize_t>(send.size()));
        std::copy(send.begin(), send.end(), sa.mutable_data());
        return py::make_tuple(sa, inv);
      },
      py::arg("keys"), py::arg("half_bits"), py::arg("n"), py::arg("pos0"), py::arg("gb"), py::arg("lb"),
      py::arg("shard_rows"), py::arg("world"), py::arg("rank"), py::arg("lo"));
  m.def("set_stream_stores", &ddl::set_stream_stores, py::arg("on"),
        "host window copies with streaming (non-temporal) stores (default on); off: plain memcpy");
  m.def("stream_stores", &ddl::stream_stores);
  m.def(
      "parallel_copy",
      [](uintptr_t dst, uintptr_t src, uint64_t bytes, int n_threads) {
        py::gil_scoped_release nogil;
        ddl::parallel_copy(reinterpret_cast<uint8_t*>(dst), reinterpret_cast<const uint8_t*>(src),
                           bytes, n_threads);
      },
      py::arg("dst"), py::arg("src"), py::arg("bytes"), py::arg("n_threads") = 4);
  m.def(
      "bind_memory_to_node",
      [](uintptr_t addr, uint64_t len, int node, bool strict) {
        return ddl::bind_memory_to_node(reinterpret_cast<void*>(addr), len, node, strict);
      },
      py::arg("addr"), py::arg("len"), py::arg("node"), py::arg("strict") = false,
      "mbind [addr, addr+len) to a NUMA node (preferred, or bound when strict; faulted pages migrate); 0 or -errno");
  m.def(
      "memory_nodes",
      [](uintptr_t addr, uint64_t len, uint64_t max_pages) {
        std::vector<int> st;
        {
          py::gil_scoped_release nogil;
          st = ddl::memory_nodes(reinterpret_cast<const void*>(addr), len, max_pages);
        }
        return st;
      },
      py::arg("addr"), py::arg("len"), py::arg("max_pages") = 64,
      "NUMA node of pages sampled over [addr, addr+len) (move_pages query; -errno per page on failure)");
  m.def(
      "pack_columns",
      [](uintptr_t dst, std::vector<uintptr_t> srcs, std::vector<uint64_t> widths, uint64_t elem_bytes, uint64_t n,
         int n_threads) {
        std::vector<const uint8_t*> ptrs;
        ptrs.reserve(srcs.size());
        for (uintptr_t a : srcs) ptrs.push_back(reinterpret_cast<const uint8_t*>(a));
        py::gil_scoped_release nogil;
        ddl::pack_columns(reinterpret_cast<uint8_t*>(dst), ptrs, widths, elem_bytes, n, n_threads);
      },
      py::arg("dst"), py::arg("srcs"), py::arg("widths"), py::arg("elem_bytes"), py::arg("n"),
      py::arg("n_threads") = 4, "k [n, w_g] column groups -> interleaved [n, sum w] (host window fill)");
  py::class_<ddl::FileHandle>(m, "RowsFile")
      .def(py::init([](const std::string& path, bool direct) {
             return std::make_unique<ddl::FileHandle>(ddl::open_rows_file(path, direct));
           }),
           py::arg("path"), py::arg("direct") = false)
      .def_property_readonly("size", [](const ddl::FileHandle& h) { return h.size; })
      .def_property_readonly("has_direct", [](const ddl::FileHandle& h) { return h.direct_fd >= 0; })
      .def_property_readonly("closed", [](const ddl::FileHandle& h) { return h.fd < 0; })
      .def("close", [](ddl::FileHandle& h) { ddl::close_rows_file(h); })
      .def(
          "read_rows",
          [](const ddl::FileHandle& h, uint64_t base_offset, uint64_t row_bytes,
             py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx, uintptr_t dst, bool direct,
             int n_threads) {
            const int64_t* ip = idx.data();
            const uint64_t n = static_cast<uint64_t>(idx.size());
            py::gil_scoped_release nogil;
            ddl::read_rows(h, base_offset, row_bytes, ip, n, reinterpret_cast<uint8_t*>(dst), direct, n_threads);
          },
          py::arg("base_offset"), py::arg("row_bytes"), py::arg("idx"), py::arg("dst"), py::arg("direct") = false,
          py::arg("n_threads") = 4, "dst[i] = row idx[i] of the file (coalesced pread, optional O_DIRECT)");
  m.def(
      "gather_ragged",
      [](uintptr_t dst, uintptr_t dst_offsets, uintptr_t src, uintptr_t src_offsets, uint64_t n_src,
         py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx, uint64_t elem_bytes, uint64_t capacity,
         int n_threads) {
        const int64_t* ip = idx.data();
        const uint64_t n = static_cast<uint64_t>(idx.size());
        py::gil_scoped_release nogil;
        return ddl::gather_ragged(reinterpret_cast<uint8_t*>(dst), reinterpret_cast<int64_t*>(dst_offsets),
                                  reinterpret_cast<const uint8_t*>(src), reinterpret_cast<const int64_t*>(src_offsets),
                                  n_src, ip, n, elem_bytes, capacity, n_threads);
      },
      py::arg("dst"), py::arg("dst_offsets"), py::arg("src"), py::arg("src_offsets"), py::arg("n_src"), py::arg("idx"),
      py::arg("elem_bytes"), py::arg("capacity"), py::arg("n_threads") = 4,
      "append sequences idx[i] of a ragged source to dst; dst_offsets[0..n] = running offsets; returns the total");
  m.def(
      "pack_plan",
      [](uintptr_t offs, int64_t n_seq, int64_t seq_len, uintptr_t row_start, uintptr_t row_end, int64_t max_rows,
         uintptr_t seg_offsets, int64_t max_segs) {
        return ddl::pack_plan(reinterpret_cast<const int64_t*>(offs), n_seq, seq_len,
                              reinterpret_cast<int64_t*>(row_start), reinterpret_cast<int64_t*>(row_end), max_rows,
                              reinterpret_cast<int64_t*>(seg_offsets), max_segs);
      },
      py::arg("offsets"), py::arg("n_seq"), py::arg("seq_len"), py::arg("row_start"), py::arg("row_end"),
      py::arg("max_rows"), py::arg("seg_offsets"), py::arg("max_segs"), "greedy in-order packing plan -> (n_rows, n_segs)");
  m.def(
      "ffd_order",
      [](py::array_t<int64_t, py::array::c_style | py::array::forcecast> lengths, int64_t seq_len) {
        const int64_t n = static_cast<int64_t>(lengths.size());
        py::array_t<int64_t> order(n);
        const int64_t rows = ddl::ffd_order(lengths.data(), n, seq_len, order.mutable_data());
        return py::make_tuple(order, rows);
      },
      py::arg("lengths"), py::arg("seq_len"),
      "first-fit-decreasing sequence order whose in-order packing breaks rows at bin ends -> (order, n_rows)");
}
