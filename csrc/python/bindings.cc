// Python bindings (pybind11) for the native runtime: the "fake JVM" host used by tests and the
// bench drives the same C ABI / engine objects a JNI host would.
#include <map>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>

#include "block_decoder.h"
#include "device_engine.h"
#include "device_ptr.h"
#include "mof_cache.h"
#include "consumer/reduce_task.h"
#include "service/merge_service.h"
#include "exchange.h"
#include "api_bench.h"
#include "generic_merger.h"
#include "j2c_sink.h"
#include "uda/aio.h"
#include "uda/codec.h"
#include "uda/datagen.h"
#include "uda/error.h"
#include "uda/hash.h"
#include "uda/ifile.h"
#include "uda/uda_bridge.h"
#include "uda/cmd.h"
#include "uda/compare.h"
#include "uda/log.h"
#include "uda/vint.h"
#include "uda/shm_group.h"
#include "uda/node_registry.h"
#include "uda/topology.h"
#include "uda/transport.h"
#include "../gpu/hbm_ledger.h"
#include <atomic>
#include <thread>

namespace py = pybind11;
using namespace uda;

namespace {

struct GpuNoise {  // start_gpu_noise / stop_gpu_noise
  std::atomic<bool> stop{false};
  std::thread thr;
  std::atomic<int64_t> ops{0};
};
GpuNoise* g_noise = nullptr;

py::dict stats_to_dict(const gpu::StepStats& s) {
  py::dict d;
  d["wall_ms"] = s.wall_ms;
  d["comm_ms"] = s.comm_ms;
  d["plan_ms"] = s.plan_ms;
  d["merge_ms"] = s.merge_ms;
  d["d2h_ms"] = s.d2h_ms;
  d["wait_out_ms"] = s.wait_out_ms;
  d["stage_ms"] = s.stage_ms;
  d["bytes_in"] = s.bytes_in;
  d["records"] = s.records;
  d["bytes_sent"] = s.bytes_sent;
  d["bytes_h2d"] = s.bytes_h2d;
  d["buffers"] = s.buffers;
  d["merge_passes"] = s.merge_passes;
  d["order_errors"] = s.order_errors;
  d["checksum"] = s.checksum;
  d["exchange_errors"] = s.exchange_errors;
  d["validated"] = s.validated;
  d["bad_layout"] = s.bad_layout;
  d["pre_merge_errors"] = s.pre_merge_errors;
  d["own_errors"] = s.own_errors;
  d["merge_errors"] = s.merge_errors;
  d["pre_d2h_errors"] = s.pre_d2h_errors;
  d["delivery_errors"] = s.delivery_errors;
  d["diag"] = s.diag;
  d["round_comm_ms"] = s.round_comm_ms;
  d["round_merge_ms"] = s.round_merge_ms;
  return d;
}

gpu::ShuffleConfig config_from_dict(const py::dict& d) {
  gpu::ShuffleConfig c;
  auto get = [&](const char* k, auto& field) {
    if (d.contains(k)) field = d[k].cast<std::decay_t<decltype(field)>>();
  };
  get("device", c.device);
  get("rank", c.rank);
  get("world", c.world);
  get("maps_per_rank", c.maps_per_rank);
  get("records_per_map", c.records_per_map);
  get("rounds", c.rounds);
  get("reducers", c.reducers);
  get("seed", c.seed);
  get("kv_buf_bytes", c.kv_buf_bytes);
  get("d2h_piece_bytes", c.d2h_piece_bytes);
  get("pinned_slots", c.pinned_slots);
  get("d2h_engines", c.d2h_engines);
  get("d2h", c.d2h);
  get("deliver_host", c.deliver_host);
  get("validate", c.validate);
  get("local_group", c.local_group);
  get("store", c.store);
  get("local_dirs", c.local_dirs);
  get("replan", c.replan);
  get("map_sort", c.map_sort);
  get("check_delivery", c.check_delivery);
  return c;
}

// Python host for the C ABI (the "fake JVM"): Python callables stand in for the UdaBridge.java
// static callbacks. Native threads take the GIL for each callback; bridge entry points release it.
struct PyBridge {
  py::object fetch_over, data_from_uda, get_path, get_conf, log, failure;
  uda_handle* h = nullptr;
  std::vector<std::shared_ptr<std::string>> keep;

  static PyBridge* self(void* ctx) { return static_cast<PyBridge*>(ctx); }
  static void t_fetch_over(void* ctx) {
    py::gil_scoped_acquire g;
    try {
      if (!self(ctx)->fetch_over.is_none()) self(ctx)->fetch_over();
    } catch (py::error_already_set& e) {
      e.discard_as_unraisable("fetch_over");
    }
  }
  static int t_data(void* ctx, const void* buf, int32_t len) {
    py::gil_scoped_acquire g;
    try {
      if (self(ctx)->data_from_uda.is_none()) return 0;
      // zero-copy like the JNI DirectByteBuffer: a read-only view valid only during the call
      py::memoryview mv = py::memoryview::from_memory(const_cast<void*>(buf), (py::ssize_t)len, true);
      py::object r = self(ctx)->data_from_uda(mv);
      mv.attr("release")();
      return r.is_none() ? 0 : r.cast<int>();
    } catch (py::error_already_set& e) {
      e.discard_as_unraisable("data_from_uda");
      return -1;
    }
  }
  static int t_get_path(void* ctx, const char* job, const char* map, int32_t reduce, uda_index_record* out) {
    py::gil_scoped_acquire g;
    try {
      if (self(ctx)->get_path.is_none()) return -1;
      py::object r = self(ctx)->get_path(std::string(job), std::string(map), reduce);
      if (r.is_none()) return -1;
      auto t = r.cast<py::tuple>();
      out->start_offset = t[0].cast<int64_t>();
      out->raw_length = t[1].cast<int64_t>();
      out->part_length = t[2].cast<int64_t>();
      std::string path = t[3].cast<std::string>();
      std::strncpy(out->path, path.c_str(), UDA_PATH_MAX - 1);
      return 0;
    } catch (py::error_already_set& e) {
      e.discard_as_unraisable("get_path");
      return -1;
    }
  }
  static int t_get_conf(void* ctx, const char* key, const char* dflt, char* out, int32_t outlen) {
    py::gil_scoped_acquire g;
    try {
      std::string v = dflt ? dflt : "";
      if (!self(ctx)->get_conf.is_none()) {
        py::object r = self(ctx)->get_conf(std::string(key), v);
        if (!r.is_none()) v = r.cast<std::string>();
      }
      int32_t n = (int32_t)std::min<size_t>(v.size(), (size_t)outlen - 1);
      std::memcpy(out, v.data(), (size_t)n);
      out[n] = 0;
      return n;
    } catch (py::error_already_set& e) {
      e.discard_as_unraisable("get_conf");
      return -1;
    }
  }
  static void t_log(void* ctx, const char* msg, int32_t sev) {
    py::gil_scoped_acquire g;
    try {
      if (!self(ctx)->log.is_none()) self(ctx)->log(std::string(msg), sev);
    } catch (py::error_already_set& e) {
      e.discard_as_unraisable("log");
    }
  }
  static void t_failure(void* ctx, const char* reason) {
    py::gil_scoped_acquire g;
    try {
      if (!self(ctx)->failure.is_none()) self(ctx)->failure(std::string(reason ? reason : ""));
    } catch (py::error_already_set& e) {
      e.discard_as_unraisable("failure");
    }
  }
  ~PyBridge() {
    if (h) {
      py::gil_scoped_release r;
      uda_destroy(h);
    }
  }
};

py::bytes cpu_merge_impl(const std::vector<std::string>& runs, const std::string& key_class, int64_t buf,
                         std::vector<int64_t>* lens) {
  KeyKind kind = key_kind_from_class(key_class.c_str());
  if (kind == KeyKind::kUnsupported) throw py::value_error("unsupported key class");
  MergeQueue q(kind);
  for (size_t i = 0; i < runs.size(); ++i) {
    auto seg = std::make_unique<MemorySegment>(reinterpret_cast<const uint8_t*>(runs[i].data()), runs[i].size());
    seg->index = (int)i;
    q.insert(std::move(seg));
  }
  KVWriter w(&q);
  std::string out;
  std::vector<uint8_t> b((size_t)buf);
  bool done = false;
  while (!done) {
    int64_t len = 0;
    done = w.fill(b.data(), buf, &len);
    out.append(reinterpret_cast<const char*>(b.data()), (size_t)len);
    lens->push_back(len);
  }
  return py::bytes(out);
}

}  // namespace

PYBIND11_MODULE(_uda_native, m) {
  m.doc() = "MI355X-native UDA shuffle/merge runtime";

  // ---------------------------------------------------------------- common
  m.def("vint_encode", [](int64_t v) {
    uint8_t b[9];
    int n = vint_encode(v, b);
    return py::bytes(reinterpret_cast<char*>(b), n);
  });
  m.def("vint_decode", [](py::bytes data) {
    std::string s = data;
    int64_t v = 0;
    int n = vint_decode(reinterpret_cast<const uint8_t*>(s.data()), s.size(), &v);
    return py::make_tuple(v, n);
  });
  m.def("vint_size", &vint_size);
  m.def("vint_decode_size", &vint_decode_size);
  m.def("parse_cmd", [](const std::string& s) {
    HadoopCmd c;
    if (!parse_cmd(s, &c)) throw py::value_error("malformed command");
    return py::make_tuple(c.count, (int)c.header, c.params);
  });
  m.def("form_cmd", &form_cmd);
  m.def("parse_options", [](const std::vector<std::string>& args) {
    NetlevOptions o;
    std::string err;
    if (!parse_options(args, &o, &err)) throw py::value_error(err);
    py::dict d;
    d["wqes_per_conn"] = o.wqes_per_conn;
    d["data_port"] = o.data_port;
    d["online"] = o.online;
    d["mode"] = o.mode;
    d["log_dir"] = o.log_dir;
    d["trace_level"] = o.trace_level;
    d["buf_size"] = o.buf_size;
    return d;
  });
  m.def("key_kind", [](const std::string& cls) { return (int)key_kind_from_class(cls.c_str()); });
  m.def("key_compare", [](int kind, py::bytes a, py::bytes b) {
    std::string sa = a, sb = b;
    return key_compare((KeyKind)kind, reinterpret_cast<const uint8_t*>(sa.data()), (int)sa.size(),
                       reinterpret_cast<const uint8_t*>(sb.data()), (int)sb.size());
  });
  m.def("record_hash", [](py::bytes b) {
    std::string s = b;
    return record_hash(reinterpret_cast<const uint8_t*>(s.data()), (int64_t)s.size());
  });
  m.def("log_set_threshold", &log_set_threshold);

  m.def("version", &uda_version);

  // ---------------------------------------------------------------- codecs
  m.def("snappy_compress", [](py::bytes b) {
    std::string s = b;
    std::string out(snappy_max_compressed_length(s.size()), '\0');
    size_t n = snappy_compress((const uint8_t*)s.data(), s.size(), (uint8_t*)&out[0]);
    out.resize(n);
    return py::bytes(out);
  });
  m.def("snappy_decompress", [](py::bytes b, size_t cap) {
    std::string s = b;
    std::string out(cap, '\0');
    size_t n = 0;
    if (!snappy_decompress((const uint8_t*)s.data(), s.size(), (uint8_t*)&out[0], cap, &n))
      throw py::value_error("corrupt snappy data");
    out.resize(n);
    return py::bytes(out);
  });
  m.def("lzo1x_compress", [](py::bytes b) {
    std::string s = b;
    std::string out(lzo1x_max_compressed_length(s.size()), '\0');
    size_t n = lzo1x_compress((const uint8_t*)s.data(), s.size(), (uint8_t*)&out[0]);
    out.resize(n);
    return py::bytes(out);
  });
  m.def("lzo1x_decompress", [](py::bytes b, size_t cap) {
    std::string s = b;
    std::string out(cap, '\0');
    size_t n = 0;
    if (!lzo1x_decompress((const uint8_t*)s.data(), s.size(), (uint8_t*)&out[0], cap, &n))
      throw py::value_error("corrupt lzo1x data");
    out.resize(n);
    return py::bytes(out);
  });
  m.def("codec_from_class", [](const std::string& c) {
    bool unsup = false;
    int v = (int)codec_from_class(c, &unsup);
    return unsup ? -1 : v;
  });
  m.def("block_compress", [](int codec, py::bytes b, size_t block) {
    std::string s = b;
    auto v = block_compress((Codec)codec, (const uint8_t*)s.data(), s.size(), block);
    return py::bytes((const char*)v.data(), v.size());
  });
  m.def("block_decompress", [](int codec, py::bytes b, size_t feed_chunk) {
    std::string s = b;
    BlockDecoder d((Codec)codec);
    std::string out;
    std::vector<uint8_t> tmp(1 << 16);
    for (size_t off = 0; off < s.size(); off += feed_chunk) {
      d.feed((const uint8_t*)s.data() + off, std::min(feed_chunk, s.size() - off));
      for (;;) {
        size_t n = d.read(tmp.data(), tmp.size());
        if (!n) break;
        out.append((const char*)tmp.data(), n);
      }
    }
    if (!d.idle()) throw py::value_error("truncated block stream");
    return py::bytes(out);
  });

  m.def("generate_runs", [](const std::string& kind, int maps, int reducers, int64_t rows, uint64_t seed) {
    std::vector<std::vector<std::vector<uint8_t>>> r;
    {
      py::gil_scoped_release g;
      r = generate_runs(kind, maps, reducers, rows, seed);
    }
    py::list out;
    for (auto& m : r) {
      py::list parts;
      for (auto& p : m) parts.append(py::bytes((const char*)p.data(), p.size()));
      out.append(parts);
    }
    return out;
  });

  // ---------------------------------------------------------------- CPU engine
  m.def("cpu_merge", [](const std::vector<std::string>& runs, const std::string& key_class, int64_t buf) {
    std::vector<int64_t> lens;
    py::bytes out = cpu_merge_impl(runs, key_class, buf, &lens);
    return py::make_tuple(out, lens);
  });

  // teravalidate: framing + order + checksum of a delivered stream, fed buffer by buffer
  py::class_<StreamValidator, std::shared_ptr<StreamValidator>>(m, "StreamValidator")
      .def(py::init([](const std::string& key_class) {
        KeyKind kind = key_kind_from_class(key_class.c_str());
        if (kind == KeyKind::kUnsupported) throw py::value_error("unsupported key class");
        return std::make_shared<StreamValidator>(kind);
      }))
      .def("feed", [](StreamValidator& v, py::buffer b) {
        py::buffer_info bi = b.request();
        v.feed(static_cast<const uint8_t*>(bi.ptr), (size_t)(bi.size * bi.itemsize));
      })
      .def_readonly("records", &StreamValidator::records)
      .def_readonly("bytes", &StreamValidator::bytes)
      .def_readonly("buffers", &StreamValidator::buffers)
      .def_readonly("order_errors", &StreamValidator::order_errors)
      .def_readonly("framing_errors", &StreamValidator::framing_errors)
      .def_readonly("checksum", &StreamValidator::checksum)
      .def_readonly("eof", &StreamValidator::eof);
  // True iff the whole-record buffer's last record is the EOF marker (-1, -1): walks the VInt framing
  // from the buffer's start (a dataFromUda buffer begins on a record boundary), so record bytes that
  // happen to end in 0xFF 0xFF are not taken for the marker. -1 on broken framing.
  m.def("buffer_ends_with_eof", [](py::buffer b) {
    py::buffer_info bi = b.request();
    const uint8_t* p = static_cast<const uint8_t*>(bi.ptr);
    const int64_t n = (int64_t)(bi.size * bi.itemsize);
    int64_t off = 0;
    while (off < n) {
      int64_t kl = 0, vl = 0;
      const int a = vint_decode(p + off, (size_t)(n - off), &kl);
      if (a <= 0) return -1;
      const int c = vint_decode(p + off + a, (size_t)(n - off - a), &vl);
      if (c <= 0) return -1;
      if (kl == -1 && vl == -1) return off + a + c == n ? 1 : -1;
      if (kl < 0 || vl < 0 || off + a + c + kl + vl > n) return -1;
      off += a + c + kl + vl;
    }
    return 0;
  });
  m.def("ifile_checksum", [](py::buffer b) {
    py::buffer_info bi = b.request();
    int64_t recs = 0, bytes = 0;
    uint64_t ck;
    {
      py::gil_scoped_release r;
      ck = ifile_checksum(static_cast<const uint8_t*>(bi.ptr), (size_t)(bi.size * bi.itemsize), &recs, &bytes);
    }
    return py::make_tuple(recs, bytes, ck);
  });

  // ---------------------------------------------------------------- async IO
  m.def("aio_selftest", [](const std::string& path, int64_t size, const std::string& backend) {
    // write `size` bytes in 64 KiB pieces then read them back through the same backend
    if (!backend.empty()) setenv("UDA_AIO_BACKEND", backend.c_str(), 1);
    auto io = AsyncIO::create(AsyncIO::Options());
    unsetenv("UDA_AIO_BACKEND");
    int fd = ::open(path.c_str(), O_CREAT | O_TRUNC | O_RDWR | O_CLOEXEC, 0600);
    if (fd < 0) throw std::runtime_error("open failed");
    std::vector<uint8_t> src((size_t)size), dst((size_t)size, 0);
    for (int64_t i = 0; i < size; ++i) src[(size_t)i] = (uint8_t)(i * 131 + (i >> 9));
    std::atomic<int64_t> bad{0};
    const int64_t piece = 64 << 10;
    for (int64_t off = 0; off < size; off += piece) {
      int64_t len = std::min(piece, size - off);
      io->write(fd, off, len, src.data() + off, [&bad, len](int64_t r) { if (r != len) bad++; });
    }
    io->drain();
    for (int64_t off = 0; off < size; off += piece) {
      int64_t len = std::min(piece, size - off);
      io->read(fd, off, len, dst.data() + off, [&bad, len](int64_t r) { if (r != len) bad++; });
    }
    io->drain();
    ::close(fd);
    return py::make_tuple(std::string(io->backend()), bad.load() == 0 && src == dst);
  });

  // AIO microbenchmark (AIOHandler_test parity, src/tests/AIOHandler_test.cc:244-249): read `size`
  // bytes of `path` in `block` pieces with up to `depth` in flight through AsyncIO (O_DIRECT when
  // `direct`), then with a sequential pread loop; returns MB/s of both.
  m.def("aio_bench", [](const std::string& path, int64_t size, int64_t block, int depth, bool direct,
                        const std::string& backend) {
    py::gil_scoped_release rel;
    {
      int fd = ::open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY | O_CLOEXEC, 0600);
      if (fd < 0) throw std::runtime_error("open for write failed");
      std::vector<uint8_t> buf((size_t)(8 << 20));
      for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(i * 2654435761u >> 13);
      for (int64_t off = 0; off < size; off += (int64_t)buf.size()) {
        const size_t n = (size_t)std::min<int64_t>((int64_t)buf.size(), size - off);
        if (::pwrite(fd, buf.data(), n, off) != (ssize_t)n) throw std::runtime_error("pwrite failed");
      }
      ::fsync(fd);
      ::close(fd);
    }
    if (!backend.empty()) setenv("UDA_AIO_BACKEND", backend.c_str(), 1);
    AsyncIO::Options o;
    o.queue_depth = std::max(depth, 1);
    auto io = AsyncIO::create(o);
    unsetenv("UDA_AIO_BACKEND");
    int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC | (direct ? O_DIRECT : 0));
    if (fd < 0 && direct) fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);  // tmpfs: no O_DIRECT
    if (fd < 0) throw std::runtime_error("open for read failed");
    const int nbuf = std::max(depth, 1);
    std::vector<void*> bufs;
    for (int i = 0; i < nbuf; ++i) bufs.push_back(aligned_alloc_io((size_t)block));
    std::atomic<int64_t> bad{0}, got{0};
    auto t0 = std::chrono::steady_clock::now();
    int64_t off = 0;
    while (off < size) {
      for (int i = 0; i < nbuf && off < size; ++i, off += block)
        io->read(fd, off, std::min(block, size - off), bufs[(size_t)i], [&](int64_t r) {
          if (r < 0) bad++;
          else got += r;
        });
      io->drain();
    }
    const double aio_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // the same reads with `depth` kept in flight throughout (a new read as each one lands), the way a
    // store loader streams a file; the batch loop above idles the device at every batch's tail
    double cont_s = 0;
    {
      std::mutex m;
      std::condition_variable cv;
      std::vector<int> free_bufs;
      for (int i = 0; i < nbuf; ++i) free_bufs.push_back(i);
      const auto c0 = std::chrono::steady_clock::now();
      for (int64_t o3 = 0; o3 < size; o3 += block) {
        int bi;
        {
          std::unique_lock<std::mutex> lk(m);
          cv.wait(lk, [&] { return !free_bufs.empty(); });
          bi = free_bufs.back();
          free_bufs.pop_back();
        }
        io->read(fd, o3, std::min(block, size - o3), bufs[(size_t)bi], [&, bi](int64_t r) {
          if (r < 0) bad++;
          std::lock_guard<std::mutex> g(m);
          free_bufs.push_back(bi);
          cv.notify_all();
        });
      }
      io->drain();
      cont_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
    }
    t0 = std::chrono::steady_clock::now();
    int64_t seq = 0;
    for (int64_t o2 = 0; o2 < size; o2 += block) {
      const ssize_t r = ::pread(fd, bufs[0], (size_t)std::min(block, size - o2), o2);
      if (r <= 0) break;
      seq += r;
    }
    const double seq_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    ::close(fd);
    for (void* b : bufs) aligned_free_io(b);
    ::unlink(path.c_str());
    py::gil_scoped_acquire acq;
    py::dict d;
    d["backend"] = std::string(io->backend());
    d["ok"] = bad.load() == 0 && got.load() == size && seq == size;
    d["aio_mbps"] = size / aio_s / 1e6;
    d["aio_streaming_mbps"] = size / cont_s / 1e6;
    d["sequential_mbps"] = size / seq_s / 1e6;
    return d;
  }, py::arg("path"), py::arg("size"), py::arg("block") = 1 << 20, py::arg("depth") = 16, py::arg("direct") = true,
     py::arg("backend") = "");

  // The provider store's read pattern without the store: `files` files of `file_bytes` written and synced,
  // then read round-robin in `chunk` pieces with `depth` reads kept in flight (O_DIRECT), as a loader
  // streams a job's MOF files. Returns GB/s; the files are removed.
  m.def("device_guard_violations", [] { return uda::gpu::device_guard_violations(); });
  // tests / tools: n idle streams on `device` kept alive until release_idle_streams() (mimics a process
  // whose pooled streams are alive: they change how new streams map onto the hardware queues)
  // tests / tools: a thread keeping `streams` extra streams of this process busy with device copies (and
  // optionally a small kernel) until stop_gpu_noise(): other streams' work sharing the hardware queues
  m.def("start_gpu_noise", [](int device, int streams, int64_t bytes) {
    if (g_noise) return;
    g_noise = new GpuNoise();
    GpuNoise* nz = g_noise;
    nz->thr = std::thread([nz, device, streams, bytes] {
      try {
        HIP_CHECK(hipSetDevice(device));
        std::vector<hipStream_t> ss(streams);
        for (auto& st : ss) HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        gpu::DeviceBuffer a((size_t)bytes * streams), b((size_t)bytes * streams);
        while (!nz->stop.load()) {
          for (int i = 0; i < streams; ++i)
            HIP_CHECK(hipMemcpyAsync(b.as<uint8_t>() + (size_t)i * bytes, a.as<uint8_t>() + (size_t)i * bytes,
                                     (size_t)bytes, hipMemcpyDeviceToDevice, ss[i]));
          for (auto& st : ss) HIP_CHECK(hipStreamSynchronize(st));
          nz->ops.fetch_add(streams);
        }
        for (auto& st : ss) (void)hipStreamDestroy(st);
      } catch (const std::exception& e) {
        UDA_LOG(kError, "gpu noise: %s", e.what());
      }
    });
  });
  m.def("stop_gpu_noise", [] {
    if (!g_noise) return (int64_t)0;
    g_noise->stop = true;
    {
      py::gil_scoped_release rel;
      if (g_noise->thr.joinable()) g_noise->thr.join();
    }
    const int64_t n = g_noise->ops.load();
    delete g_noise;
    g_noise = nullptr;
    return n;
  });
  // node topology (uda/topology.h): every GPU of the node with its NUMA node and consumer CPU slice
  // (UDA_SYSFS_ROOT lets a test describe any node); `allowed` empty = no affinity restriction
  m.def("topology_plan", [](const std::vector<int>& allowed) {
    py::list out;
    const auto gpus = node_gpus();
    for (const auto& g : gpus) {
      py::dict d;
      d["bdf"] = g.bdf();
      d["numa_node"] = g.numa_node;
      d["cpus"] = consumer_cpus(g, gpus, allowed);
      out.append(d);
    }
    return out;
  }, py::arg("allowed") = std::vector<int>());
  m.def("lzo_lane_decode_host", [](py::bytes stream, int64_t raw_cap) {
    const std::string in = stream;
    std::string out((size_t)std::max<int64_t>(raw_cap, 1), '\0');
    int64_t n = 0;
    if (!gpu::lzo_lane_decode_host(reinterpret_cast<const uint8_t*>(in.data()), (int64_t)in.size(),
                                   reinterpret_cast<uint8_t*>(&out[0]), raw_cap, &n))
      throw std::runtime_error("lzo lane decode: corrupt block");
    out.resize((size_t)n);
    return py::bytes(out);
  });
  m.def("usable_gpu_bdfs", [] {
    std::vector<std::string> v;
    for (const auto& g : usable_gpus()) v.push_back(g.bdf());
    return v;
  });
  m.def("format_cpulist", &format_cpulist);
  m.def("parse_cpulist", &parse_cpulist);
  // a rank's placement record (bench.py JSON): PCI address, NUMA node, consumer CPU slice
  m.def("device_placement", [](int device) {
    py::dict d;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) == hipSuccess) d["pci"] = std::string(bus);
    d["numa_node"] = gpu::device_numa_node(device);
    d["consumer_cpus"] = format_cpulist(gpu::device_consumer_cpus(device));
    return d;
  });
  // hipDeviceCanAccessPeer over the visible devices: m[i][j] (diagonal 1)
  m.def("peer_access_matrix", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    std::vector<std::vector<int>> m2((size_t)n, std::vector<int>((size_t)n, 0));
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        int can = i == j ? 1 : 0;
        if (i != j && hipDeviceCanAccessPeer(&can, i, j) != hipSuccess) can = -1;
        m2[(size_t)i][(size_t)j] = can;
      }
    return m2;
  });
  m.def("hold_idle_streams", [](int device, int n, int priority) {
    static std::vector<hipStream_t>& held = *new std::vector<hipStream_t>();
    HIP_CHECK(hipSetDevice(device));
    for (int i = 0; i < n; ++i) {
      hipStream_t s = nullptr;
      HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
      held.push_back(s);
    }
    return (int)held.size();
  }, py::arg("device"), py::arg("n"), py::arg("priority") = 0);

  m.def("aio_interleave_bench", [](const std::string& dir, int files, int64_t file_bytes, int64_t chunk, int depth) {
    py::gil_scoped_release rel;
    file_bytes = file_bytes / chunk * chunk;
    std::vector<std::string> paths;
    std::vector<int> fds;
    {
      std::vector<uint8_t> buf((size_t)(8 << 20));
      for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(i * 2654435761u >> 13);
      for (int f = 0; f < files; ++f) {
        paths.push_back(dir + "/uda_interleave." + std::to_string(getpid()) + "." + std::to_string(f));
        const int fd = ::open(paths.back().c_str(), O_CREAT | O_TRUNC | O_WRONLY | O_CLOEXEC, 0600);
        if (fd < 0) throw std::runtime_error("open for write failed");
        for (int64_t off = 0; off < file_bytes; off += (int64_t)buf.size())
          if (::pwrite(fd, buf.data(), (size_t)std::min<int64_t>((int64_t)buf.size(), file_bytes - off), off) <= 0)
            throw std::runtime_error("pwrite failed");
        ::fdatasync(fd);
        ::close(fd);
      }
    }
    for (const auto& p : paths) {
      int fd = ::open(p.c_str(), O_RDONLY | O_CLOEXEC | O_DIRECT);
      if (fd < 0) fd = ::open(p.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) throw std::runtime_error("open for read failed");
      fds.push_back(fd);
    }
    AsyncIO::Options o;
    o.queue_depth = std::max(depth, 1) * 2;
    auto io = AsyncIO::create(o);
    std::vector<void*> bufs;
    for (int i = 0; i < depth; ++i) bufs.push_back(aligned_alloc_io((size_t)chunk));
    std::mutex m;
    std::condition_variable cv;
    std::vector<int> free_bufs;
    for (int i = 0; i < depth; ++i) free_bufs.push_back(i);
    std::atomic<int64_t> bad{0};
    const auto t0 = std::chrono::steady_clock::now();
    for (int64_t off = 0; off < file_bytes; off += chunk)
      for (int f = 0; f < files; ++f) {
        int bi;
        {
          std::unique_lock<std::mutex> lk(m);
          cv.wait(lk, [&] { return !free_bufs.empty(); });
          bi = free_bufs.back();
          free_bufs.pop_back();
        }
        io->read(fds[(size_t)f], off, chunk, bufs[(size_t)bi], [&, bi](int64_t r) {
          if (r < 0) bad++;
          std::lock_guard<std::mutex> g(m);
          free_bufs.push_back(bi);
          cv.notify_all();
        });
      }
    io->drain();
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int fd : fds) ::close(fd);
    for (void* b : bufs) aligned_free_io(b);
    for (const auto& p : paths) ::unlink(p.c_str());
    if (bad.load()) throw std::runtime_error("interleaved read failed");
    return (double)file_bytes * files / secs / 1e9;
  }, py::arg("dir"), py::arg("files"), py::arg("file_bytes"), py::arg("chunk") = 16 << 20, py::arg("depth") = 16);

  // ---------------------------------------------------------------- bridge (C ABI)
  py::class_<PyBridge, std::shared_ptr<PyBridge>>(m, "Bridge")
      .def(py::init([](bool is_net_merger, const std::vector<std::string>& args, int log_level, py::object fetch_over,
                       py::object data_from_uda, py::object get_path, py::object get_conf, py::object log,
                       py::object failure) {
             auto b = std::make_shared<PyBridge>();
             b->fetch_over = fetch_over;
             b->data_from_uda = data_from_uda;
             b->get_path = get_path;
             b->get_conf = get_conf;
             b->log = log;
             b->failure = failure;
             uda_callbacks cb;
             std::memset(&cb, 0, sizeof(cb));
             cb.ctx = b.get();
             cb.fetch_over = &PyBridge::t_fetch_over;
             cb.data_from_uda = &PyBridge::t_data;
             cb.get_path = &PyBridge::t_get_path;
             cb.get_conf = &PyBridge::t_get_conf;
             cb.log = log.is_none() ? nullptr : &PyBridge::t_log;
             cb.failure = &PyBridge::t_failure;
             std::vector<const char*> argv;
             for (auto& a : args) argv.push_back(a.c_str());
             {
               py::gil_scoped_release r;
               b->h = uda_start(is_net_merger ? 1 : 0, (int)argv.size(), argv.data(), log_level, 0, &cb);
             }
             if (!b->h) throw std::runtime_error("uda_start failed");
             return b;
           }),
           py::arg("is_net_merger"), py::arg("args"), py::arg("log_level") = 3, py::arg("fetch_over") = py::none(),
           py::arg("data_from_uda") = py::none(), py::arg("get_path") = py::none(), py::arg("get_conf") = py::none(),
           py::arg("log") = py::none(), py::arg("failure") = py::none())
      .def("do_command",
           [](PyBridge& b, const std::string& cmd) {
             int r;
             {
               py::gil_scoped_release g;
               r = uda_do_command(b.h, cmd.c_str());
             }
             if (r != 0) throw std::runtime_error(std::string("UdaRuntimeException: ") + uda_last_error(b.h));
           })
      .def("reduce_exit",
           [](PyBridge& b) {
             py::gil_scoped_release g;
             return uda_reduce_exit(b.h);
           })
      .def("register_mof",
           [](PyBridge& b, const std::string& job, const std::string& map, py::bytes data,
              const std::vector<int64_t>& index) {
             // the bridge keeps a reference: the data must outlive the provider
             auto keep = std::make_shared<std::string>(data);
             b.keep.push_back(keep);
             return uda_provider_register_mof(b.h, job.c_str(), map.c_str(), keep->data(), (int64_t)keep->size(),
                                              index.data(), (int32_t)(index.size() / 3));
           })
      .def("register_mof_device",
           [](PyBridge& b, const std::string& job, const std::string& map, uintptr_t dev_ptr, int64_t len,
              const std::vector<int64_t>& index, int device) {
             return uda_provider_register_mof_device(b.h, job.c_str(), map.c_str(), reinterpret_cast<const void*>(dev_ptr),
                                                     len, index.data(), (int32_t)(index.size() / 3), device);
           })
      .def("stats", [](PyBridge& b) { return uda_stats_string(b.h); });
  // node-local shared-memory control plane of the IPC exchange (CPU-testable, no HIP)
  py::class_<ShmGroup>(m, "ShmGroup")
      .def(py::init<const std::string&, int, int, size_t, size_t, double>(), py::arg("name"), py::arg("rank"),
           py::arg("world"), py::arg("mailbox_bytes") = 1 << 16, py::arg("outbox_bytes") = 1 << 16,
           py::arg("timeout_s") = 60.0, py::call_guard<py::gil_scoped_release>())
      .def("barrier", [](ShmGroup& g) { g.barrier("python"); }, py::call_guard<py::gil_scoped_release>())
      .def("try_barrier", &ShmGroup::try_barrier, py::call_guard<py::gil_scoped_release>())
      .def("abort", &ShmGroup::abort)
      .def("aborted", &ShmGroup::aborted)
      .def("abort_reason", &ShmGroup::abort_reason)
      .def("publish", [](ShmGroup& g, int c, int64_t v) { g.publish((ShmGroup::Counter)c, v); })
      .def("read", [](ShmGroup& g, int c, int peer) { return g.read((ShmGroup::Counter)c, peer); })
      .def("wait_at_least",
           [](ShmGroup& g, int c, int peer, int64_t v) { g.wait_at_least((ShmGroup::Counter)c, peer, v, "python"); },
           py::call_guard<py::gil_scoped_release>())
      .def("alltoall",
           [](ShmGroup& g, const std::vector<int64_t>& send) {
             if (send.size() % (size_t)g.world()) throw std::runtime_error("alltoall: size not a multiple of world");
             std::vector<int64_t> recv(send.size());
             {
               py::gil_scoped_release nogil;
               g.alltoall_i64(send.data(), recv.data(), send.size() / (size_t)g.world());
             }
             return recv;
           })
      .def("publish_alloc",
           [](ShmGroup& g, py::bytes b, int64_t size) {
             const std::string s = b;
             return g.publish_alloc(s.data(), s.size(), size);
           })
      .def("read_alloc", [](ShmGroup& g, int peer, int id) -> py::object {
        char blob[ShmGroup::kAllocBlob];
        int64_t size = 0;
        if (!g.read_alloc(peer, id, blob, sizeof(blob), &size)) return py::none();
        return py::make_tuple(py::bytes(blob, sizeof(blob)), size);
      });

  // node-local registry of reduce tasks / HBM bytes per GPU (CPU-testable, no HIP)
  py::class_<NodeRegistry>(m, "NodeRegistry")
      .def(py::init<const std::string&>(), py::arg("name") = std::string())
      .def_property_readonly("name", &NodeRegistry::name)
      .def("place_task",
           [](NodeRegistry& r, const std::vector<std::string>& keys, const std::string& tag) {
             const NodeRegistry::Placement p = r.place_task(keys, tag);
             return py::make_tuple(p.index, p.slot);
           })
      .def("add_task", &NodeRegistry::add_task)
      .def("release", &NodeRegistry::release)
      .def("set_bytes", &NodeRegistry::set_bytes, py::arg("key"), py::arg("bytes"), py::arg("resident") = 0)
      .def("usage",
           [](NodeRegistry& r, const std::string& key) {
             const NodeRegistry::Use u = r.usage(key);
             py::dict d;
             d["tasks"] = u.tasks;
             d["bytes"] = u.bytes;
             d["resident"] = u.resident;
             return d;
           })
      .def_property_readonly("reclaimed", &NodeRegistry::reclaimed)
      .def("unlink", &NodeRegistry::unlink);
  m.def("process_running", &process_running, py::arg("pid"), py::arg("start") = 0);
  m.def("process_start_ticks", &process_start_ticks);
  // HBM budget ledger on fake devices (no HIP): tests of admission, trimming and the node-wide total
  m.def("hbm_fake_device", [](int d, int64_t total, const std::string& key) {
    gpu::HbmLedger::get().set_fake_device(d, total, key);
  });
  m.def("hbm_fake_untracked", [](int d, int64_t b) { gpu::HbmLedger::get().set_fake_untracked(d, b); });
  m.def("hbm_configure", [](int d, double conf) { gpu::HbmLedger::get().configure(d, conf); });
  m.def("hbm_alloc", [](int d, int64_t b, bool resident) { gpu::HbmLedger::get().on_alloc(d, b, resident); },
        py::arg("device"), py::arg("bytes"), py::arg("resident") = false);
  m.def("hbm_free", [](int d, int64_t b, bool resident) { gpu::HbmLedger::get().on_free(d, b, resident); },
        py::arg("device"), py::arg("bytes"), py::arg("resident") = false);
  m.def("hbm_headroom", [](int d) { return gpu::HbmLedger::get().headroom(d); });
  m.def("hbm_stats", [](int d) {
    const gpu::HbmLedger::Stats s = gpu::HbmLedger::get().stats(d);
    py::dict o;
    o["budget"] = s.budget;
    o["used"] = s.used;
    o["reserved"] = s.reserved;
    o["peak"] = s.peak;
    o["resident"] = s.resident;
    o["node_bytes"] = s.node_bytes;
    o["trimmed"] = s.trimmed;
    o["over"] = s.over;
    o["waits"] = s.waits;
    o["wait_ms"] = s.wait_ms;
    o["device_peak"] = s.device_peak;
    return o;
  });
  // an idle pool of fake objects: trimmed by the ledger under pressure (returns the pool's id)
  m.def("hbm_fake_pool", [](int d, std::vector<int64_t> sizes) {
    auto objs = std::make_shared<std::vector<int64_t>>(std::move(sizes));
    auto mu = std::make_shared<std::mutex>();
    for (int64_t b : *objs) gpu::HbmLedger::get().on_alloc(d, b);
    gpu::HbmLedger::get().add_pool(
        {[objs, mu, d](int dev, int64_t want) -> int64_t {
           if (dev != d) return 0;
           std::vector<int64_t> drop;
           {
             std::lock_guard<std::mutex> g(*mu);
             std::sort(objs->begin(), objs->end());
             int64_t got = 0;
             while (!objs->empty() && got < want) {
               got += objs->back();
               drop.push_back(objs->back());
               objs->pop_back();
             }
           }
           int64_t freed = 0;
           for (int64_t b : drop) {
             gpu::HbmLedger::get().on_free(d, b);
             freed += b;
           }
           return freed;
         },
         [objs, mu, d](int dev) -> int64_t {
           if (dev != d) return 0;
           std::lock_guard<std::mutex> g(*mu);
           int64_t n = 0;
           for (int64_t b : *objs) n += b;
           return n;
         }});
  });
  struct PyReservation {
    std::unique_ptr<gpu::HbmLedger::Reservation> r;
  };
  py::class_<PyReservation, std::shared_ptr<PyReservation>>(m, "HbmReservation")
      .def_property_readonly("granted", [](PyReservation& p) { return p.r ? p.r->granted() : 0; })
      .def_property_readonly("wait_ms", [](PyReservation& p) { return p.r ? p.r->wait_ms() : 0.0; })
      .def("alloc", [](PyReservation& p, int64_t b) {  // an allocation drawing from the reservation
        if (!p.r) throw std::runtime_error("reservation released");
        auto scope = p.r->bind();
        gpu::HbmLedger::get().on_alloc(p.r->device(), b);
      })
      .def("release", [](PyReservation& p) { p.r.reset(); });
  m.def("hbm_reserve",
        [](int d, int64_t bytes, double timeout_s) {
          auto p = std::make_shared<PyReservation>();
          {
            py::gil_scoped_release nogil;
            p->r = gpu::HbmLedger::get().reserve(d, bytes, nullptr, timeout_s);
            // the Python thread is not where the allocations happen: unbind (alloc() binds per call)
            p->r->unbind();
          }
          return p;
        },
        py::arg("device"), py::arg("bytes"), py::arg("timeout_s") = 30.0);

  m.def("set_log_level", &uda_set_log_level);

  // ---------------------------------------------------------------- GPU engine
  // the provider's HBM store of MOF files on its own (gpu/mof_cache.h): loads, holders, eviction
  py::class_<gpu::MofCache>(m, "MofStore")
      .def(py::init([](int64_t capacity, std::vector<int> devices, double lease_s, int64_t chunk_bytes,
                       double idle_evict_s, bool cached_read) {
             gpu::MofCache::Options o;
             o.capacity = capacity;
             o.devices = devices;
             o.lease_s = lease_s;
             o.chunk_bytes = chunk_bytes;
             o.idle_evict_s = idle_evict_s;
             o.cached_read = cached_read;
             return new gpu::MofCache(o);
           }),
           py::arg("capacity"), py::arg("devices") = std::vector<int>{0}, py::arg("lease_s") = 600.0,
           py::arg("chunk_bytes") = 16 << 20, py::arg("idle_evict_s") = 0.0, py::arg("cached_read") = true)
      .def("acquire",
           [](gpu::MofCache& c, const std::string& job, const std::string& path, const std::string& holder) {
             gpu::MofCache::Ref r;
             std::string why;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = c.acquire(job, path, holder, &r, &why);
             }
             return py::make_tuple(ok, why, (uint64_t)(uintptr_t)r.data, r.len, r.device);
           })
      .def("release", &gpu::MofCache::release)
      .def("release_holder", &gpu::MofCache::release_holder)
      .def("job_over", &gpu::MofCache::job_over)
      .def("stats", [](gpu::MofCache& c) {
        const gpu::MofCache::Stats s = c.stats();
        py::dict d;
        d["loads"] = s.loads;
        d["hits"] = s.hits;
        d["declined"] = s.declined;
        d["evictions"] = s.evictions;
        d["bytes_loaded"] = s.bytes_loaded;
        d["resident_bytes"] = s.resident_bytes;
        d["holders"] = s.holders;
        d["holders_reaped"] = s.holders_reaped;
        d["releases"] = s.releases;
        d["cached_reads"] = s.cached_reads;
        return d;
      });
  m.def("reducer_holder_id", &gpu::reducer_holder_id);
  // the merge service's peer-credential rule (mapred.uda.gpu.merge.service.users)
  m.def("merge_service_user_allowed", [](const std::string& users, int uid) {
    return MergeService::user_allowed(users, (uid_t)uid);
  });
  m.def("merge_service_default_path", &MergeService::default_path);
  // fetch throughput of the TCP transport alone: every listed partition fetched whole into one buffer,
  // `maps_at_once` partitions at a time with `depth` requests of `chunk` bytes in flight each
  m.def("tcp_fetch_probe", [](const std::string& host, int port, const std::string& job,
                              const std::vector<std::string>& maps, int reduce, const std::vector<int64_t>& sizes,
                              int64_t chunk, int depth, int connections, int maps_at_once) {
    auto nogil = std::make_unique<py::gil_scoped_release>();
    auto cl = make_tcp_client(port, 256, connections);
    int64_t total = 0;
    std::vector<int64_t> base(maps.size() + 1, 0);
    for (size_t i = 0; i < maps.size(); ++i) base[i + 1] = base[i] + sizes[i];
    total = base.back();
    std::unique_ptr<uint8_t[]> buf(new uint8_t[(size_t)std::max<int64_t>(total, 1)]);
    std::mutex m;
    std::condition_variable cv;
    std::string err;
    const auto t0 = std::chrono::steady_clock::now();
    std::atomic<size_t> next_map{0};
    std::vector<std::thread> ts;
    for (int w = 0; w < std::max(1, maps_at_once); ++w)
      ts.emplace_back([&] {
        for (size_t i; (i = next_map++) < maps.size();) {
          int inflight = 0;
          int64_t at = 0;
          std::unique_lock<std::mutex> lk(m);
          while (at < sizes[i] || inflight > 0) {
            while (at < sizes[i] && inflight < depth && err.empty()) {
              FetchRequest rq;
              rq.job_id = job;
              rq.map_id = maps[i];
              rq.reduce_id = reduce;
              rq.fetched = at;
              rq.buf_len = std::min(chunk, sizes[i] - at);
              at += rq.buf_len;
              ++inflight;
              lk.unlock();
              cl->fetch(host, rq, buf.get() + base[i] + rq.fetched, [&](const FetchAck& a) {
                std::lock_guard<std::mutex> g(m);
                if (a.status != 0 && err.empty()) err = a.error;
                --inflight;
                cv.notify_all();
              });
              lk.lock();
            }
            if (!err.empty() && inflight == 0) break;
            cv.wait(lk, [&] { return inflight == 0 || (at < sizes[i] && inflight < depth && err.empty()); });
            if (!err.empty() && inflight == 0) break;
          }
        }
      });
    for (auto& t : ts) t.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    cl->close();
    uint64_t sum = 0;
    for (int64_t k = 0; k < total; k += 4096) sum += buf[(size_t)k];
    nogil.reset();  // the GIL again before any Python object is made
    if (!err.empty()) throw std::runtime_error("tcp_fetch_probe: " + err);
    return py::make_tuple(total, s, sum);
  });
  // one TCP client, a fetch to an unreachable host on one thread and, while it is still trying, one to a
  // live host: returns (live fetch ms, dead host error, dead host ms, second dead fetch ms)
  m.def("mof_host_is_local", &uda::mof_host_is_local);
  m.def("local_mof_readable", [](const std::string& path, int64_t off, int64_t len) {
    const int fd = uda::open_local_mof(path, off, len);
    if (fd >= 0) ::close(fd);
    return fd >= 0;
  });
  // ACK string codec (transport.h): format then parse, as a TCP reducer sees the provider's answer
  m.def("ack_roundtrip", [](int status, int64_t raw_len, int64_t part_len, int64_t sent, int64_t mof_offset,
                            const std::string& path, const std::string& error) {
    uda::FetchAck a;
    a.status = status;
    a.raw_len = raw_len;
    a.part_len = part_len;
    a.sent = sent;
    a.mof_offset = mof_offset;
    a.path = path;
    a.error = error;
    uda::FetchAck b;
    if (!uda::parse_ack(uda::format_ack(a), &b)) throw std::runtime_error("ack does not parse");
    py::dict d;
    d["status"] = b.status;
    d["raw_len"] = b.raw_len;
    d["part_len"] = b.part_len;
    d["sent"] = b.sent;
    d["mof_offset"] = b.mof_offset;
    d["path"] = b.path;
    d["error"] = b.error;
    return d;
  });
  m.def("tcp_dead_host_probe", [](const std::string& live, const std::string& dead, int port, const std::string& job,
                                  const std::string& map, int reduce, int64_t size) {
    py::gil_scoped_release rel;
    auto cl = make_tcp_client(port, 256, 4);
    std::unique_ptr<uint8_t[]> a(new uint8_t[(size_t)std::max<int64_t>(size, 1)]), b(new uint8_t[64]);
    auto fetch = [&](const std::string& host, uint8_t* dst, int64_t len, std::string* err) {
      std::mutex m;
      std::condition_variable cv;
      bool done = false;
      FetchRequest rq;
      rq.job_id = job;
      rq.map_id = map;
      rq.reduce_id = reduce;
      rq.buf_len = len;
      const auto t0 = std::chrono::steady_clock::now();
      cl->fetch(host, rq, dst, [&](const FetchAck& k) {
        std::lock_guard<std::mutex> g(m);
        if (k.status != 0) *err = k.error.empty() ? "status " + std::to_string(k.status) : k.error;
        done = true;
        cv.notify_all();
      });
      std::unique_lock<std::mutex> lk(m);
      cv.wait(lk, [&] { return done; });
      return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };
    std::string dead_err, live_err, dead2_err;
    double dead_ms = 0;
    std::thread t([&] { dead_ms = fetch(dead, b.get(), 64, &dead_err); });
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    const double live_ms = fetch(live, a.get(), size, &live_err);
    t.join();
    const double dead2_ms = fetch(dead, b.get(), 64, &dead2_err);
    cl->close();
    if (!live_err.empty()) throw std::runtime_error("live host fetch failed: " + live_err);
    return std::make_tuple(live_ms, dead_err, dead_ms, dead2_ms);
  });
  m.def("open_ipc_mappings", &gpu::open_ipc_mappings);
  m.def("device_read", [](uint64_t addr, int64_t len) {  // device bytes back to the host (tests)
    std::string out((size_t)len, '\0');
    if (len > 0) HIP_CHECK(hipMemcpy(out.data(), reinterpret_cast<const void*>((uintptr_t)addr), (size_t)len,
                                     hipMemcpyDeviceToHost));
    return py::bytes(out);
  });
  m.def("device_count", &gpu::device_count);
  m.def("ipc_safe_bytes", [](uint64_t b) { return (uint64_t)gpu::ipc_safe_bytes((size_t)b); });
  m.def("ipc_size_ok", [](uint64_t b) { return gpu::ipc_size_ok((size_t)b); });
  m.def("node_id", []() { return gpu::node_id(); });
  // (address or None, reason): what a reducer does with a provider's descriptor
  m.def("descriptor_resolve", [](const std::string& desc, int device) -> py::tuple {
    std::string why;
    const uint8_t* p = gpu::try_resolve_device_descriptor(desc, device, &why);
    if (!p) return py::make_tuple(py::none(), why);
    return py::make_tuple((uint64_t)(uintptr_t)p, why);
  });
  m.def("descriptor_make", [](int device, uint64_t addr, const std::string& handle_hex, uint64_t base) {
    gpu::IpcExport ex;
    ex.handle_hex = handle_hex;
    ex.base = reinterpret_cast<const uint8_t*>((uintptr_t)base);
    return gpu::make_device_descriptor(device, reinterpret_cast<const uint8_t*>((uintptr_t)addr), ex);
  });
  // N8 device discovery: per-pair P2P reachability, link type (HSA_AMD_LINK_INFO_TYPE_*: 2 = xGMI) and
  // hop count, and the runtime's relative performance rank.
  m.def("device_topology", []() {
    py::dict d;
    int n = gpu::device_count();
    d["devices"] = n;
    py::list props, links;
    for (int i = 0; i < n; ++i) {
      hipDeviceProp_t p;
      if (hipGetDeviceProperties(&p, i) != hipSuccess) continue;
      py::dict e;
      e["name"] = std::string(p.name);
      e["arch"] = std::string(p.gcnArchName);
      e["cus"] = p.multiProcessorCount;
      e["hbm_bytes"] = (int64_t)p.totalGlobalMem;
      e["lds_bytes"] = (int64_t)p.sharedMemPerBlock;
      e["l2_bytes"] = p.l2CacheSize;
      e["pci_bus"] = p.pciBusID;
      props.append(e);
      for (int j = 0; j < n; ++j) {
        if (i == j) continue;
        int can = 0, rank = -1;
        uint32_t type = 0, hops = 0;
        (void)hipDeviceCanAccessPeer(&can, i, j);
        (void)hipDeviceGetP2PAttribute(&rank, hipDevP2PAttrPerformanceRank, i, j);
        (void)hipExtGetLinkTypeAndHopCount(i, j, &type, &hops);
        py::dict l;
        l["src"] = i;
        l["dst"] = j;
        l["p2p"] = can != 0;
        l["link_type"] = type;
        l["hops"] = hops;
        l["perf_rank"] = rank;
        links.append(l);
      }
    }
    d["props"] = props;
    d["links"] = links;
    return d;
  });
  // Merge IFile runs (any bytes-like objects, read in place) on the device. Returns
  // (merged bytes, buffer cuts, records, merge passes, device merge ms, runs indexed serially).
  m.def("gpu_merge_runs", [](const py::list& runs, const std::string& key_class, int64_t kv_buf, int device) {
    KeyKind kind = key_kind_from_class(key_class.c_str());
    if (kind == KeyKind::kUnsupported) throw py::value_error("unsupported key class");
    std::vector<py::buffer_info> views;
    std::vector<const uint8_t*> host;
    std::vector<int64_t> bytes;
    int64_t total = 0;
    for (auto h : runs) {
      views.push_back(py::reinterpret_borrow<py::buffer>(h).request());
      host.push_back(static_cast<const uint8_t*>(views.back().ptr));
      bytes.push_back((int64_t)(views.back().size * views.back().itemsize));
      total += bytes.back();
    }
    std::vector<int64_t> cuts;
    int64_t records = 0, out_bytes = 0;
    int passes = 0, serial_runs = 0;
    double merge_ms = 0;
    gpu::DeviceBuffer in, dout;
    hipStream_t s = nullptr;
    {
      py::gil_scoped_release rel;
      HIP_CHECK(hipSetDevice(device));
      in.alloc((size_t)std::max<int64_t>(total, 16));
      dout.alloc((size_t)std::max<int64_t>(total, 16));
      HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      std::vector<const uint8_t*> ptrs;
      int64_t off = 0;
      for (size_t i = 0; i < host.size(); ++i) {
        if (bytes[i]) HIP_CHECK(hipMemcpyAsync(in.as<uint8_t>() + off, host[i], (size_t)bytes[i], hipMemcpyHostToDevice, s));
        ptrs.push_back(in.as<uint8_t>() + off);
        off += bytes[i];
      }
      // one merger (and its HBM workspace) per device for the process, like the NetMerger's pooled
      // DeviceWorkspace: a reducer process merges many times, so only the first call allocates
      static std::mutex gm_mu;
      static auto* gm_cache = new std::map<int, std::unique_ptr<gpu::GenericMerger>>();  // outlives HIP at exit
      std::unique_lock<std::mutex> gm_lock(gm_mu);
      auto& gm_slot = (*gm_cache)[device];
      if (!gm_slot) gm_slot.reset(new gpu::GenericMerger());
      gpu::GenericMerger& gm = *gm_slot;
      HIP_CHECK(hipStreamSynchronize(s));
      auto t0 = std::chrono::steady_clock::now();
      auto res = gm.merge(ptrs, bytes, (int)kind, dout.as<uint8_t>(), total, kv_buf, s);
      HIP_CHECK(hipStreamSynchronize(s));
      merge_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      cuts = res.cuts;
      records = res.records;
      passes = res.passes;
      out_bytes = res.bytes;
      serial_runs = gm.f1_serial_runs();
    }
    views.clear();
    // the result is copied D2H straight into the bytes object's storage
    PyObject* o = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)out_bytes);
    if (!o) throw py::error_already_set();
    py::bytes out = py::reinterpret_steal<py::bytes>(o);
    {
      py::gil_scoped_release rel;
      if (out_bytes) HIP_CHECK(hipMemcpyAsync(PyBytes_AS_STRING(o), dout.as(), (size_t)out_bytes, hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
      HIP_CHECK(hipStreamDestroy(s));
      in.reset();
      dout.reset();
    }
    return py::make_tuple(out, cuts, records, passes, merge_ms, serial_runs);
  }, py::arg("runs"), py::arg("key_class"), py::arg("kv_buf") = 1 << 20, py::arg("device") = 0);
  // F8: sort TeraSort records (104-byte IFile records, no EOF marker) by their 10-byte key on the
  // device; returns (sorted bytes, device ms of the sort).
  m.def("gpu_sort_fixed", [](py::buffer b, int device, bool staged) {
    py::buffer_info v = b.request();
    const int64_t bytes = (int64_t)(v.size * v.itemsize);
    if (bytes % gpu::kTeraRecordBytes) throw py::value_error("not a whole number of 104-byte records");
    const int64_t n = bytes / gpu::kTeraRecordBytes;
    if (n >= (int64_t)UINT32_MAX) throw py::value_error("too many records");
    PyObject* o = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)bytes);
    if (!o) throw py::error_already_set();
    py::bytes out = py::reinterpret_steal<py::bytes>(o);
    float ms = 0;
    {
      py::gil_scoped_release rel;
      HIP_CHECK(hipSetDevice(device));
      gpu::DeviceBuffer d, ws;
      d.alloc((size_t)std::max<int64_t>(bytes + 2, 16));
      ws.alloc((size_t)gpu::sort_fixed_ws_bytes(std::max<int64_t>(n, 1)));
      hipStream_t s = nullptr;
      hipEvent_t e0 = nullptr, e1 = nullptr;
      HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      HIP_CHECK(hipEventCreate(&e0));
      HIP_CHECK(hipEventCreate(&e1));
      // staged: input in the workspace's record area, sorted run gathered into d (+ EOF marker)
      uint8_t* in = staged ? gpu::sort_fixed_ws_records(ws.as(), std::max<int64_t>(n, 1)) : d.as<uint8_t>();
      if (bytes) HIP_CHECK(hipMemcpyAsync(in, v.ptr, (size_t)bytes, hipMemcpyHostToDevice, s));
      gpu::launch_sort_fixed_run(d.as<uint8_t>(), n, ws.as(), s, staged);  // warm-up (first launch loads code)
      if (bytes) HIP_CHECK(hipMemcpyAsync(in, v.ptr, (size_t)bytes, hipMemcpyHostToDevice, s));
      HIP_CHECK(hipEventRecord(e0, s));
      gpu::launch_sort_fixed_run(d.as<uint8_t>(), n, ws.as(), s, staged);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipEventRecord(e1, s));
      if (bytes) HIP_CHECK(hipMemcpyAsync(PyBytes_AS_STRING(o), d.as(), (size_t)bytes, hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      (void)hipStreamDestroy(s);
    }
    return py::make_tuple(out, (double)ms);
  }, py::arg("records"), py::arg("device") = 0, py::arg("staged") = false);
  // F6: decode Hadoop block-compressed streams on the device; returns (raw streams, blocks, decode_ms)
  m.def("gpu_block_decode", [](const std::string& codec_cls, const std::vector<std::string>& streams, int device) {
    bool unsup = false;
    Codec c = codec_from_class(codec_cls, &unsup);
    if (c == Codec::kNone) c = codec_cls == "snappy" ? Codec::kSnappy : codec_cls == "lzo" ? Codec::kLzo : Codec::kNone;
    if (c == Codec::kNone) throw py::value_error("unknown codec " + codec_cls);
    std::vector<std::string> outs;
    int64_t blocks = 0;
    double ms = 0;
    {
      py::gil_scoped_release rel;
      HIP_CHECK(hipSetDevice(device));
      std::vector<const uint8_t*> ptrs;
      std::vector<int64_t> lens;
      int64_t staged = 0;
      for (auto& st : streams) {
        ptrs.push_back(reinterpret_cast<const uint8_t*>(st.data()));
        lens.push_back((int64_t)st.size());
        staged += (int64_t)st.size();
      }
      gpu::BlockPlan plan;
      if (!gpu::plan_block_streams(c, ptrs, lens, &plan)) throw UdaError("block framing not resolvable on device");
      gpu::DeviceBuffer din((size_t)std::max<int64_t>(staged, 16)), dout((size_t)std::max<int64_t>(plan.raw_total, 16));
      hipStream_t s;
      HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      int64_t off = 0;
      for (auto& st : streams) {
        if (!st.empty()) HIP_CHECK(hipMemcpyAsync(din.as<uint8_t>() + off, st.data(), st.size(), hipMemcpyHostToDevice, s));
        off += (int64_t)st.size();
      }
      HIP_CHECK(hipStreamSynchronize(s));
      gpu::DeviceBlockDecoder dec;
      auto t0 = std::chrono::steady_clock::now();
      dec.decode(c, plan, din.as<uint8_t>(), dout.as<uint8_t>(), s);
      ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      std::string all((size_t)plan.raw_total, '\0');
      if (plan.raw_total) HIP_CHECK(hipMemcpyAsync(&all[0], dout.as(), all.size(), hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
      HIP_CHECK(hipStreamDestroy(s));
      for (size_t i = 0; i < streams.size(); ++i)
        outs.push_back(all.substr((size_t)plan.raw_offset[i], (size_t)(plan.raw_offset[i + 1] - plan.raw_offset[i])));
      blocks = (int64_t)plan.descs.size();
    }
    py::list l;
    for (auto& o : outs) l.append(py::bytes(o));
    return py::make_tuple(l, blocks, ms);
  }, py::arg("codec"), py::arg("streams"), py::arg("device") = 0);
  m.def("nccl_unique_id", []() { return py::bytes(gpu::nccl_unique_id()); });
  // RCCL data-plane self test on one GPU: communicator bootstrap from an ncclUniqueId and the grouped
  // send/recv counts exchange the shuffle plan uses (world 1: the rank exchanges with itself).
  m.def("rccl_selftest", [](int device, int n) {
    py::gil_scoped_release rel;
    HIP_CHECK(hipSetDevice(device));
    auto ex = gpu::make_rccl_exchange(0, 1, gpu::nccl_unique_id());
    hipStream_t s;
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<int64_t> send((size_t)n), recv((size_t)n, -1);
    for (int i = 0; i < n; ++i) send[(size_t)i] = (int64_t)i * 1000003 - 7;
    ex->alltoall_i64(send.data(), recv.data(), (size_t)n, s);
    HIP_CHECK(hipStreamDestroy(s));
    return std::string(ex->name()) + (send == recv ? ":ok" : ":mismatch");
  }, py::arg("device") = 0, py::arg("n") = 4096);

  // Exchange backends with hand-made plans (tests): the local group runs its ranks as threads here;
  // the IPC probe is one rank (call it from one process per rank).
  m.def("local_exchange_probe",
        [](int world, const std::vector<std::vector<std::vector<int64_t>>>& send,
           const std::vector<std::vector<std::vector<int64_t>>>& recv, bool host_source, int rounds, int device) {
          py::gil_scoped_release rel;
          static std::atomic<int> gen{0};
          const std::string name = "probe" + std::to_string(gen++);
          std::vector<std::string> out(world);
          std::vector<std::thread> ts;
          for (int r = 0; r < world; ++r)
            ts.emplace_back([&, r] {
              try {
                HIP_CHECK(hipSetDevice(device));
                auto ex = gpu::make_local_exchange(name, r, world);
                out[r] = gpu::exchange_probe(*ex, device, send.at(r), recv.at(r), host_source, rounds);
              } catch (const std::exception& e) {
                out[r] = e.what();
              }
            });
          for (auto& t : ts) t.join();
          return out;
        },
        py::arg("world"), py::arg("send"), py::arg("recv"), py::arg("host_source") = false, py::arg("rounds") = 1,
        py::arg("device") = 0);
  m.def("ipc_exchange_probe",
        [](const std::string& name, int rank, int world, const std::vector<std::vector<int64_t>>& send,
           const std::vector<std::vector<int64_t>>& recv, bool host_source, int rounds, int device,
           int64_t export_bytes) {
          py::gil_scoped_release rel;
          try {
            HIP_CHECK(hipSetDevice(device));
            auto ex = gpu::make_ipc_exchange(name, rank, world, device);
            return gpu::exchange_probe(*ex, device, send, recv, host_source, rounds, export_bytes);
          } catch (const std::exception& e) {
            return std::string(e.what());
          }
        },
        py::arg("name"), py::arg("rank"), py::arg("world"), py::arg("send"), py::arg("recv"),
        py::arg("host_source") = false, py::arg("rounds") = 1, py::arg("device") = 0, py::arg("export_bytes") = 0);

  py::class_<gpu::J2CSink, std::shared_ptr<gpu::J2CSink>>(m, "J2CSink")
      .def(py::init([](int r, int64_t kv, py::object threaded) {
             return std::make_shared<gpu::J2CSink>(r, kv, threaded.is_none() ? gpu::J2CSink::default_threaded()
                                                                               : threaded.cast<bool>());
           }),
           py::arg("reducers"), py::arg("kv_buf_bytes") = 1 << 20, py::arg("threaded") = py::none())
      .def_property_readonly("reducers", &gpu::J2CSink::reducers)
      .def_property_readonly("threaded", &gpu::J2CSink::threaded)
      .def("flush", &gpu::J2CSink::flush, py::call_guard<py::gil_scoped_release>())
      .def("records", &gpu::J2CSink::records)
      .def("bytes", &gpu::J2CSink::bytes)
      .def("buffers", &gpu::J2CSink::buffers)
      .def("eof", &gpu::J2CSink::eof)
      .def("error", &gpu::J2CSink::error)
      .def("order_errors", &gpu::J2CSink::order_errors)
      .def("set_check_order", &gpu::J2CSink::set_check_order)
      .def("reset", &gpu::J2CSink::reset, py::call_guard<py::gil_scoped_release>())
      // one dataFromUda buffer for reducer r (returns the sink's status code, 0 = ok); reps > 1
      // consumes the same buffer again (micro-benchmarks; EOF buffers only once)
      .def("consume", [](gpu::J2CSink& s, int r, py::buffer b, int reps) {
        py::buffer_info bi = b.request();
        const auto* p = static_cast<const uint8_t*>(bi.ptr);
        const int64_t n = (int64_t)(bi.size * bi.itemsize);
        if (r < 0 || r >= s.reducers()) throw py::index_error("reducer out of range");
        py::gil_scoped_release rel;
        int rc = 0;
        for (int i = 0; i < std::max(1, reps) && rc == 0; ++i) rc = s.consume(r, p, n);
        return rc;
      }, py::arg("reducer"), py::arg("data"), py::arg("reps") = 1);

  py::class_<gpu::ApiTeraSortBench>(m, "ApiTeraSortBench")
      .def(py::init([](const py::dict& d) {
        gpu::ApiBenchConfig c;
        auto get = [&](const char* k, auto& field) {
          if (d.contains(k)) field = d[k].cast<std::decay_t<decltype(field)>>();
        };
        get("device", c.device);
        get("maps", c.maps);
        get("reducers", c.reducers);
        get("records_per_map", c.records_per_map);
        get("seed", c.seed);
        get("kv_buf_bytes", c.kv_buf_bytes);
        get("round_bytes", c.round_bytes);
        get("rank", c.rank);
        get("world", c.world);
        get("port", c.port);
        get("transport", c.transport);
        get("bind_addr", c.bind_addr);
        get("host_mofs", c.host_mofs);
        get("fetch", c.fetch);
        get("max_concurrent_merges", c.max_concurrent_merges);
        get("provider_workers", c.provider_workers);
        get("mof_dir", c.mof_dir);
        get("provider_hbm_bytes", c.provider_hbm_bytes);
        get("workload", c.workload);
        get("skew", c.skew);
        get("codec", c.codec);
        return new gpu::ApiTeraSortBench(c);
      }))
      .def("setup", &gpu::ApiTeraSortBench::setup, py::call_guard<py::gil_scoped_release>())
      .def("step",
           [](gpu::ApiTeraSortBench& b, bool validate) {
             std::string info;
             std::map<std::string, double> r;
             {
               py::gil_scoped_release g;
               r = b.step(validate, &info);
             }
             py::dict d;
             for (auto& kv : r) d[kv.first.c_str()] = kv.second;
             d["task0_stats"] = info;
             return d;
           },
           py::arg("validate") = false)
      .def("expected_records", &gpu::ApiTeraSortBench::expected_records)
      .def("provider_stats", &gpu::ApiTeraSortBench::provider_stats)
      .def_property_readonly("compressed_bytes", &gpu::ApiTeraSortBench::compressed_bytes)
      .def("local_partition_records", &gpu::ApiTeraSortBench::local_partition_records)
      .def("set_expected", &gpu::ApiTeraSortBench::set_expected)
      .def("set_peers", &gpu::ApiTeraSortBench::set_peers)
      .def("task_commands", &gpu::ApiTeraSortBench::task_commands)
      .def("provider_port", &gpu::ApiTeraSortBench::provider_port)
      .def_property_readonly("store_bytes", &gpu::ApiTeraSortBench::store_bytes);

  py::class_<gpu::ShuffleJob>(m, "ShuffleJob")
      .def(py::init([](const py::dict& cfg) { return new gpu::ShuffleJob(config_from_dict(cfg)); }))
      // std::string, not py::bytes: the argument is converted while the GIL is held (a py::bytes would
      // be read and released inside the GIL-free call)
      .def("init_comm", [](gpu::ShuffleJob& j, const std::string& uid) { j.init_comm(uid); },
           py::call_guard<py::gil_scoped_release>())
      .def("init_local", &gpu::ShuffleJob::init_local, py::call_guard<py::gil_scoped_release>())
      .def("init_ipc", &gpu::ShuffleJob::init_ipc, py::call_guard<py::gil_scoped_release>())
      .def("generate", &gpu::ShuffleJob::generate, py::call_guard<py::gil_scoped_release>())
      .def("sample_keys",
           [](gpu::ShuffleJob& j, int64_t every) {
             auto v = j.sample_keys(every);
             py::list out;
             for (auto& d : v) {
               py::array_t<uint64_t> a({(py::ssize_t)(d.size() / 2), (py::ssize_t)2});
               if (!d.empty()) std::memcpy(a.mutable_data(), d.data(), d.size() * 8);
               out.append(a);
             }
             return out;
           })
      .def("set_bounds",
           [](gpu::ShuffleJob& j, py::array_t<uint64_t, py::array::c_style> b) {
             std::vector<uint64_t> v(b.data(), b.data() + b.size());
             j.set_bounds(v);
           })
      .def("plan", &gpu::ShuffleJob::plan, py::call_guard<py::gil_scoped_release>())
      .def("set_j2c_sink",
           [](gpu::ShuffleJob& j, std::shared_ptr<gpu::J2CSink> s) {
             if (s->reducers() != j.config().reducers) throw py::value_error("J2CSink reducer count mismatch");
             j.set_sink([s](int r, const uint8_t* buf, int64_t len) { return s->consume(r, buf, len); });
           })
      .def("set_python_sink",
           [](gpu::ShuffleJob& j, py::function fn, bool with_reducer) {
             auto holder = std::make_shared<py::function>(fn);
             j.set_sink([holder, with_reducer](int r, const uint8_t* buf, int64_t len) {
               py::gil_scoped_acquire g;
               try {
                 py::bytes b(reinterpret_cast<const char*>(buf), (size_t)len);
                 py::object res = with_reducer ? (*holder)(r, b) : (*holder)(b);
                 return res.is_none() ? 0 : res.cast<int>();
               } catch (py::error_already_set& e) {
                 e.discard_as_unraisable("ShuffleJob python sink");
                 return -1;
               }
             });
           },
           py::arg("fn"), py::arg("with_reducer") = false)
      .def("clear_sink", [](gpu::ShuffleJob& j) { j.set_sink(nullptr); })
      .def("run_step",
           [](gpu::ShuffleJob& j, bool validate) {
             gpu::StepStats st;
             {
               py::gil_scoped_release r;
               st = j.run_step(validate);
             }
             return stats_to_dict(st);
           },
           py::arg("validate") = false)
      .def("reducer_records", &gpu::ShuffleJob::reducer_records)
      .def_property_readonly("comm_ranks", &gpu::ShuffleJob::comm_ranks)
      .def_property_readonly("exchange_name", &gpu::ShuffleJob::exchange_name)
      .def_property_readonly("delivery_name", &gpu::ShuffleJob::delivery_name)
      .def_property_readonly("store_name", &gpu::ShuffleJob::store_name)
      .def("local_dest_checksums", &gpu::ShuffleJob::local_dest_checksums)
      .def("local_dest_records", &gpu::ShuffleJob::local_dest_records)
      .def("index_record", &gpu::ShuffleJob::index_record)
      .def("read_partition",
           [](gpu::ShuffleJob& j, int mp, int d) {
             auto v = j.read_partition(mp, d);
             return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
           })
      .def("mof_device_ptr", [](gpu::ShuffleJob& j, int m) { return (uintptr_t)j.mof_device_ptr(m); })
      .def("mof_bytes", &gpu::ShuffleJob::mof_bytes)
      .def_property_readonly("store_bytes", &gpu::ShuffleJob::store_bytes)
      .def_property_readonly("map_sort_ms", &gpu::ShuffleJob::map_sort_ms)
      .def_property_readonly("max_round_records", &gpu::ShuffleJob::max_round_records)
      .def("peer_send_bytes", &gpu::ShuffleJob::peer_send_bytes);
}
