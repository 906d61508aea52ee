// NetMerger GPU backend (mapred.uda.merge.backend=gpu): every fetched MOF partition is staged in
// HBM and the whole reduce input is merged by the generic HIP merge tree (csrc/gpu/generic.hip),
// then streamed back to the host reducer through dataFromUda in whole-record buffers.
//
// Reference counterpart: merge_online (src/Merger/MergeManager.cc:184-193) — the same fetch and
// progress semantics, with the heap merge replaced by the device merge.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <random>
#include <thread>

#include "../gpu/device_engine.h"
#include "../gpu/generic_merger.h"
#include "reduce_task.h"
#include "uda/log.h"

namespace uda {

void ReduceTask::merge_gpu() {
  if (gpu::device_count() <= 0) throw UdaError("mapred.uda.merge.backend=gpu but no HIP device is visible");
  auto t0 = std::chrono::steady_clock::now();
  const int maps = init_.num_maps;
  const int device = (int)host_->conf_i64("mapred.uda.gpu.device", 0);
  if (hipSetDevice(device) != hipSuccess) throw UdaError("hipSetDevice failed");

  // ---- fetch: start every MOF (bounded by the buffer pool), drain each fully into host memory
  std::vector<std::vector<uint8_t>> parts;
  std::mt19937_64 rng((uint64_t)std::chrono::steady_clock::now().time_since_epoch().count());
  int started = 0, drained = 0;
  std::vector<FetchParams> pending;
  std::vector<std::shared_ptr<MofFetcher>> ready;
  while (drained < maps) {
    std::vector<std::shared_ptr<MofFetcher>> to_start;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] {
        return stop_ || !fetched_.empty() || ((!fetch_list_.empty() || !pending.empty()) && free_pairs_ > 0 && started < maps);
      });
      if (stop_) throw UdaError("reduce task stopped during fetch");
      while (!fetch_list_.empty()) {
        pending.push_back(fetch_list_.front());
        fetch_list_.pop_front();
      }
      std::shuffle(pending.begin(), pending.end(), rng);
      while (!pending.empty() && free_pairs_ > 0 && started < maps) {
        to_start.push_back(std::make_shared<MofFetcher>(this, pending.back(), buffer_size_, codec_));
        pending.pop_back();
        free_pairs_--;
        started++;
      }
      while (!fetched_.empty()) {
        ready.push_back(fetched_.front());
        fetched_.pop_front();
      }
    }
    for (auto& f : to_start) f->start();
    // drain arrived MOFs in parallel (each drain keeps one request in flight ahead)
    std::vector<std::vector<uint8_t>> got(ready.size());
    std::vector<std::exception_ptr> errs(ready.size());
    std::vector<std::thread> ts;
    for (size_t i = 0; i < ready.size(); ++i)
      ts.emplace_back([&, i] {
        try {
          std::vector<uint8_t> buf((size_t)buffer_size_);
          for (;;) {
            int64_t n = ready[i]->pull(buf.data(), (int64_t)buf.size());
            if (n == 0) break;
            got[i].insert(got[i].end(), buf.begin(), buf.begin() + n);
          }
        } catch (...) {
          errs[i] = std::current_exception();
        }
      });
    for (auto& t : ts) t.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
    for (auto& g : got) {
      parts.push_back(std::move(g));
      drained++;
      progress_count_++;
      total_count_++;
      {
        std::lock_guard<std::mutex> gl(st_mu_);
        st_.maps_fetched++;
      }
      if (progress_count_ == 20 || total_count_ == maps) {
        host_->fetch_over();
        progress_count_ = 0;
      }
    }
    ready.clear();
  }
  const double fetch_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();

  // ---- stage in HBM and merge
  int64_t total = 0;
  for (auto& p : parts) total += (int64_t)p.size();
  gpu::DeviceBuffer in((size_t)std::max<int64_t>(total, 16)), out((size_t)std::max<int64_t>(total, 16));
  std::vector<const uint8_t*> runs;
  std::vector<int64_t> bytes;
  int64_t off = 0;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) throw UdaError("hipStreamCreate failed");
  for (auto& p : parts) {
    if (!p.empty()) HIP_CHECK(hipMemcpyAsync(in.as<uint8_t>() + off, p.data(), p.size(), hipMemcpyHostToDevice, s));
    runs.push_back(in.as<uint8_t>() + off);
    bytes.push_back((int64_t)p.size());
    off += (int64_t)p.size();
  }
  gpu::GenericMerger merger;
  gpu::GenericMergeResult r = merger.merge(runs, bytes, (int)kind_, out.as<uint8_t>(), total, kv_buf_size_ - kEofBytes, s);
  std::vector<uint8_t> host((size_t)r.bytes + kEofBytes);
  if (r.bytes) HIP_CHECK(hipMemcpyAsync(host.data(), out.as(), (size_t)r.bytes, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  (void)hipStreamDestroy(s);
  host[(size_t)r.bytes] = 0xFF;
  host[(size_t)r.bytes + 1] = 0xFF;

  // ---- deliver: buffers at the device-computed cuts; EOF rides in the last one
  for (size_t j = 0; j + 1 < r.cuts.size(); ++j) {
    if (stop_) throw UdaError("reduce task stopped during merge");
    const int64_t b = r.cuts[j], e = r.cuts[j + 1];
    const bool last = (j + 2 == r.cuts.size());
    const int64_t len = (e - b) + (last ? kEofBytes : 0);
    if (host_->data_from_uda(host.data() + b, (int32_t)len) != 0) throw UdaError("dataFromUda callback failed");
    std::lock_guard<std::mutex> g(st_mu_);
    st_.buffers++;
    st_.bytes_delivered += len;
  }
  if (r.cuts.size() < 2) {  // empty reduce input: EOF only
    if (host_->data_from_uda(host.data() + r.bytes, kEofBytes) != 0) throw UdaError("dataFromUda callback failed");
    std::lock_guard<std::mutex> g(st_mu_);
    st_.buffers++;
    st_.bytes_delivered += kEofBytes;
  }
  std::lock_guard<std::mutex> g(st_mu_);
  st_.records += r.records;
  st_.fetch_ms = fetch_ms;
  st_.merge_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() - fetch_ms;
}

}  // namespace uda
