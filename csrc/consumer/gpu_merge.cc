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

#include "../gpu/block_decoder.h"
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
  // F6: compressed partitions cross PCIe compressed and are decoded in HBM (host decode only when
  // the framing needs it, see plan_block_streams)
  const bool device_decode = codec_ != Codec::kNone && host_->conf_i64("mapred.uda.gpu.decompress", 1) != 0;
  const Codec fetch_codec = device_decode ? Codec::kNone : codec_;

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
        to_start.push_back(std::make_shared<MofFetcher>(this, pending.back(), buffer_size_, fetch_codec));
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

  // ---- stage in HBM (decoding compressed partitions there) and merge
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) throw UdaError("hipStreamCreate failed");
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } stream_guard{s};
  gpu::BlockPlan plan;
  bool decode_on_device = false;
  if (device_decode) {
    std::vector<const uint8_t*> ptrs;
    std::vector<int64_t> lens;
    for (auto& p : parts) {
      ptrs.push_back(p.data());
      lens.push_back((int64_t)p.size());
    }
    decode_on_device = gpu::plan_block_streams(codec_, ptrs, lens, &plan);
    if (!decode_on_device) {
      UDA_LOG(kInfo, "device decode: framing needs a host decode (multi-chunk %s block); decoding on host",
              codec_name(codec_));
      for (auto& p : parts) {
        BlockDecoder dec(codec_);
        dec.feed(p.data(), p.size());
        std::vector<uint8_t> raw, buf(1 << 20);
        for (size_t n; (n = dec.read(buf.data(), buf.size())) > 0;) raw.insert(raw.end(), buf.begin(), buf.begin() + (long)n);
        if (!dec.idle()) throw UdaError("truncated compressed partition");
        p.swap(raw);
      }
    }
  }
  int64_t total = 0, staged = 0;
  for (auto& p : parts) staged += (int64_t)p.size();
  total = decode_on_device ? plan.raw_total : staged;
  gpu::DeviceBuffer in((size_t)std::max<int64_t>(total, 16)), out((size_t)std::max<int64_t>(total, 16));
  gpu::DeviceBuffer packed(decode_on_device ? (size_t)std::max<int64_t>(staged, 16) : 0);
  uint8_t* stage = decode_on_device ? packed.as<uint8_t>() : in.as<uint8_t>();
  std::vector<const uint8_t*> runs;
  std::vector<int64_t> bytes;
  int64_t off = 0;
  for (size_t i = 0; i < parts.size(); ++i) {
    auto& p = parts[i];
    if (!p.empty()) HIP_CHECK(hipMemcpyAsync(stage + off, p.data(), p.size(), hipMemcpyHostToDevice, s));
    if (decode_on_device) {
      runs.push_back(in.as<uint8_t>() + plan.raw_offset[i]);
      bytes.push_back(plan.raw_offset[i + 1] - plan.raw_offset[i]);
    } else {
      runs.push_back(in.as<uint8_t>() + off);
      bytes.push_back((int64_t)p.size());
    }
    off += (int64_t)p.size();
  }
  if (decode_on_device) {
    gpu::DeviceBlockDecoder dec;
    dec.decode(codec_, plan, packed.as<uint8_t>(), in.as<uint8_t>(), s);
    std::lock_guard<std::mutex> g(st_mu_);
    st_.device_decoded_blocks += (int64_t)plan.descs.size();
  }
  gpu::GenericMerger merger;
  gpu::GenericMergeResult r = merger.merge(runs, bytes, (int)kind_, out.as<uint8_t>(), total, kv_buf_size_ - kEofBytes, s);
  std::vector<uint8_t> host((size_t)r.bytes + kEofBytes);
  if (r.bytes) HIP_CHECK(hipMemcpyAsync(host.data(), out.as(), (size_t)r.bytes, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  parts.clear();
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
