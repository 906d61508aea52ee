// Python bindings (pybind11) for the native runtime: the "fake JVM" host used by tests and the
// bench drives the same C ABI / engine objects a JNI host would.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <cstring>

#include "device_engine.h"
#include "uda/cmd.h"
#include "uda/compare.h"
#include "uda/log.h"
#include "uda/vint.h"

namespace py = pybind11;
using namespace uda;

namespace {

py::dict stats_to_dict(const gpu::StepStats& s) {
  py::dict d;
  d["wall_ms"] = s.wall_ms;
  d["split_ms"] = s.split_ms;
  d["comm_ms"] = s.comm_ms;
  d["merge_ms"] = s.merge_ms;
  d["d2h_ms"] = s.d2h_ms;
  d["bytes_in"] = s.bytes_in;
  d["records"] = s.records;
  d["bytes_sent"] = s.bytes_sent;
  d["buffers"] = s.buffers;
  d["merge_passes"] = s.merge_passes;
  d["order_errors"] = s.order_errors;
  d["checksum"] = s.checksum;
  d["bad_layout"] = s.bad_layout;
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
  get("seed", c.seed);
  get("kv_buf_bytes", c.kv_buf_bytes);
  get("d2h_piece_bytes", c.d2h_piece_bytes);
  get("pinned_slots", c.pinned_slots);
  get("d2h_streams", c.d2h_streams);
  get("deliver_host", c.deliver_host);
  get("validate", c.validate);
  return c;
}

// Native sink that counts bytes and buffers (the bench's reducer stand-in: it receives the
// merged stream zero-copy, as J2CQueue would after its memcpy).
struct CountingSink {
  std::atomic<int64_t> bytes{0};
  std::atomic<int64_t> buffers{0};
  std::atomic<int64_t> max_len{0};
};

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
    return gpu::record_hash(reinterpret_cast<const uint8_t*>(s.data()), (int64_t)s.size());
  });
  m.def("log_set_threshold", &log_set_threshold);

  // ---------------------------------------------------------------- GPU engine
  m.def("device_count", &gpu::device_count);
  m.def("nccl_unique_id", []() { return py::bytes(gpu::nccl_unique_id()); });

  py::class_<CountingSink, std::shared_ptr<CountingSink>>(m, "CountingSink")
      .def(py::init<>())
      .def_property_readonly("bytes", [](CountingSink& s) { return s.bytes.load(); })
      .def_property_readonly("buffers", [](CountingSink& s) { return s.buffers.load(); })
      .def_property_readonly("max_len", [](CountingSink& s) { return s.max_len.load(); })
      .def("reset", [](CountingSink& s) {
        s.bytes = 0;
        s.buffers = 0;
        s.max_len = 0;
      });

  py::class_<gpu::ShuffleJob>(m, "ShuffleJob")
      .def(py::init([](const py::dict& cfg) { return new gpu::ShuffleJob(config_from_dict(cfg)); }))
      .def("init_comm", [](gpu::ShuffleJob& j, py::bytes uid) { j.init_comm(uid); },
           py::call_guard<py::gil_scoped_release>())
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
      .def("set_counting_sink",
           [](gpu::ShuffleJob& j, std::shared_ptr<CountingSink> s) {
             j.set_sink([s](const uint8_t*, int64_t len) {
               s->bytes += len;
               s->buffers += 1;
               int64_t cur = s->max_len.load();
               while (len > cur && !s->max_len.compare_exchange_weak(cur, len)) {
               }
               return 0;
             });
           })
      .def("set_python_sink",
           [](gpu::ShuffleJob& j, py::function fn) {
             auto holder = std::make_shared<py::function>(fn);
             j.set_sink([holder](const uint8_t* buf, int64_t len) {
               py::gil_scoped_acquire g;
               py::object r = (*holder)(py::bytes(reinterpret_cast<const char*>(buf), (size_t)len));
               return r.is_none() ? 0 : r.cast<int>();
             });
           })
      .def("clear_sink", [](gpu::ShuffleJob& j) { j.set_sink(nullptr); })
      .def("run_step",
           [](gpu::ShuffleJob& j) {
             gpu::StepStats s;
             {
               py::gil_scoped_release r;
               s = j.run_step();
             }
             return stats_to_dict(s);
           })
      .def("local_dest_checksums", &gpu::ShuffleJob::local_dest_checksums)
      .def("local_dest_records", &gpu::ShuffleJob::local_dest_records)
      .def("index_record", &gpu::ShuffleJob::index_record)
      .def("read_partition",
           [](gpu::ShuffleJob& j, int mp, int d) {
             auto v = j.read_partition(mp, d);
             return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
           })
      .def_property_readonly("store_bytes", &gpu::ShuffleJob::store_bytes)
      .def_property_readonly("max_round_records", &gpu::ShuffleJob::max_round_records);
}
