// uda_mof_supplier: a node's MOFSupplier as a process of its own (the NodeManager aux service /
// TaskTracker side, src/MOFServer/MOFSupplierMain.cc:87-143), holding a synthetic job's map outputs in
// its HBM and serving them over TCP: descriptor fetches answer with hipIpc handles, so the node's
// reduce task processes (uda_reduce_task) merge the partitions where they lie.
//
//   uda_mof_supplier key=value...     (device, maps, reducers, records_per_map, round_bytes, workload,
//                                      skew, codec, port, bind, workers, seed, service)
//
// service=<socket path>: the process is also the node's merge service (merge_service.h): reduce task
// processes started with mapred.uda.gpu.merge.service=<path> run their NetMerger in here.
//
// After setup it prints one JSON line: the port, the store size, every reduce task's expected record
// count and its command strings (INIT + FETCHes, as its ReduceTask JVM would send them). Then it
// serves until stdin says "exit" (or closes); "stats" prints the provider's stats as one JSON line.
// Every GPU call of the node benchmark (bench.py --api --node) happens in native processes on the
// system HIP runtime, the way a Hadoop node runs libuda.so.
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <memory>
#include <string>

#include "api_bench.h"
#include "service/merge_service.h"

namespace {
std::string js(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += (unsigned char)c < 0x20 ? ' ' : c;
  }
  return o + "\"";
}
}  // namespace

int main(int argc, char** argv) {
  uda::gpu::ApiBenchConfig c;
  c.transport = "tcp";
  c.bind_addr = "127.0.0.1";
  c.fetch = "device";
  std::string service;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    const size_t eq = a.find('=');
    if (eq == std::string::npos) {
      std::fprintf(stderr, "usage: %s key=value...\n", argv[0]);
      return 2;
    }
    const std::string k = a.substr(0, eq), v = a.substr(eq + 1);
    if (k == "device") c.device = std::atoi(v.c_str());
    else if (k == "maps") c.maps = std::atoi(v.c_str());
    else if (k == "reducers") c.reducers = std::atoi(v.c_str());
    else if (k == "records_per_map") c.records_per_map = std::atoll(v.c_str());
    else if (k == "round_bytes") c.round_bytes = std::atoll(v.c_str());
    else if (k == "workload") c.workload = v;
    else if (k == "skew") c.skew = std::atof(v.c_str());
    else if (k == "codec") c.codec = v;
    else if (k == "port") c.port = std::atoi(v.c_str());
    else if (k == "bind") c.bind_addr = v;
    else if (k == "workers") c.provider_workers = std::atoi(v.c_str());
    else if (k == "seed") c.seed = std::strtoull(v.c_str(), nullptr, 0);
    else if (k == "service") service = v;
    else {
      std::fprintf(stderr, "uda_mof_supplier: unknown key %s\n", k.c_str());
      return 2;
    }
  }
  try {
    std::unique_ptr<uda::MergeService> svc;  // first: the pinned rings allocated after it are shareable
    if (!service.empty()) svc = std::make_unique<uda::MergeService>(service);
    uda::gpu::ApiTeraSortBench b(c);
    b.setup();
    std::string out = "{\"port\":" + std::to_string(b.provider_port()) + ",\"store_bytes\":" +
                      std::to_string(b.store_bytes()) + ",\"expected\":[";
    const auto e = b.expected_records();
    for (size_t i = 0; i < e.size(); ++i) out += (i ? "," : "") + std::to_string(e[i]);
    out += "],\"commands\":[";
    for (int r = 0; r < c.reducers; ++r) {
      out += r ? ",[" : "[";
      const auto cmds = b.task_commands(r);
      for (size_t i = 0; i < cmds.size(); ++i) out += (i ? "," : "") + js(cmds[i]);
      out += "]";
    }
    out += "]}";
    std::printf("%s\n", out.c_str());
    std::fflush(stdout);
    for (std::string line; std::getline(std::cin, line);) {
      if (line == "exit") break;
      if (line == "stats") {
        std::string st = b.provider_stats();
        if (svc && !st.empty() && st.back() == '}')
          st = st.substr(0, st.size() - 1) + ",\"merge_service\":{\"sessions\":" + std::to_string(svc->sessions()) +
               ",\"zero_copy_buffers\":" + std::to_string(svc->zero_copy_buffers()) +
               ",\"bounced_buffers\":" + std::to_string(svc->bounced_buffers()) + "}}";
        std::printf("%s\n", st.c_str());
        std::fflush(stdout);
      }
    }
  } catch (const std::exception& ex) {
    std::printf("{\"error\":%s}\n", js(ex.what()).c_str());
    return 1;
  }
  return 0;
}
