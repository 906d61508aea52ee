// IFile parsing, segments, heap k-way merge and greedy buffer writer. See uda/ifile.h.
#include "uda/ifile.h"

#include <chrono>

#include "uda/error.h"

namespace uda {

Parse ifile_parse(const uint8_t* p, size_t avail, RecordView* r) {
  int64_t kl = 0, vl = 0;
  int a = vint_decode(p, avail, &kl);
  if (a == 0) return Parse::kPartial;
  int b = vint_decode(p + a, avail - a, &vl);
  if (b == 0) return Parse::kPartial;
  if (kl == kEofMarker && vl == kEofMarker) {
    r->hdr = a + b;
    r->klen = r->vlen = -1;
    return Parse::kEof;
  }
  if (kl < 0 || vl < 0 || kl > INT32_MAX || vl > INT32_MAX) return Parse::kCorrupt;
  if ((size_t)(a + b) + (size_t)kl + (size_t)vl > avail) return Parse::kPartial;
  r->hdr = a + b;
  r->key = p + a + b;
  r->klen = (int32_t)kl;
  r->val = r->key + kl;
  r->vlen = (int32_t)vl;
  return Parse::kRecord;
}

int64_t ifile_record_size(int64_t klen, int64_t vlen) {
  return vint_size(klen) + vint_size(vlen) + klen + vlen;
}

int64_t ifile_write(uint8_t* buf, const uint8_t* k, int32_t kl, const uint8_t* v, int32_t vl) {
  int64_t n = vint_encode(kl, buf);
  n += vint_encode(vl, buf + n);
  if (kl) std::memcpy(buf + n, k, (size_t)kl);
  n += kl;
  if (vl) std::memcpy(buf + n, v, (size_t)vl);
  return n + vl;
}

void ifile_append(std::vector<uint8_t>* out, const uint8_t* k, int32_t kl, const uint8_t* v, int32_t vl) {
  size_t o = out->size();
  out->resize(o + (size_t)ifile_record_size(kl, vl));
  ifile_write(out->data() + o, k, kl, v, vl);
}

void ifile_append_eof(std::vector<uint8_t>* out) {
  out->push_back(0xFF);
  out->push_back(0xFF);
}

// ---------------------------------------------------------------------------- MemorySegment
bool MemorySegment::next() {
  if (eof_) return false;
  if (pos_ >= len_) {  // tolerate streams without an explicit EOF marker
    eof_ = true;
    return false;
  }
  Parse r = ifile_parse(p_ + pos_, len_ - pos_, &cur_);
  if (r == Parse::kEof) {
    eof_ = true;
    return false;
  }
  if (r != Parse::kRecord) throw UdaError("corrupt or truncated IFile segment");
  pos_ += (size_t)cur_.size();
  ++records;
  return true;
}

// ---------------------------------------------------------------------------- StreamSegment
StreamSegment::StreamSegment(ChunkSource src, int64_t chunk_bytes)
    : src_(std::move(src)), chunk_(chunk_bytes > 64 ? chunk_bytes : 64) {
  buf_.resize((size_t)chunk_);
}

bool StreamSegment::refill() {
  if (src_done_) return false;
  // carry the unconsumed tail (a record split across chunks) to the front: the join
  const size_t tail = len_ - pos_;
  if (tail && pos_) std::memmove(buf_.data(), buf_.data() + pos_, tail);
  pos_ = 0;
  len_ = tail;
  if (len_ + (size_t)chunk_ > buf_.size()) buf_.resize(len_ + (size_t)chunk_);
  auto t0 = std::chrono::steady_clock::now();
  int64_t got = src_(buf_.data() + len_, chunk_);
  wait_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  if (got < 0) throw UdaError("segment source failed");
  if (got == 0) {
    src_done_ = true;
    return false;
  }
  len_ += (size_t)got;
  return true;
}

bool StreamSegment::next() {
  if (eof_) return false;
  for (;;) {
    Parse r = (len_ > pos_) ? ifile_parse(buf_.data() + pos_, len_ - pos_, &cur_) : Parse::kPartial;
    if (r == Parse::kRecord) {
      pos_ += (size_t)cur_.size();
      ++records;
      return true;
    }
    if (r == Parse::kEof) {
      eof_ = true;
      return false;
    }
    if (r == Parse::kCorrupt) throw UdaError("corrupt IFile stream");
    // partial: a larger record may need more than one chunk; keep growing the window
    if (!refill()) {
      if (len_ == pos_) {
        eof_ = true;
        return false;
      }
      throw UdaError("IFile stream truncated inside a record");
    }
  }
}

// ---------------------------------------------------------------------------- MergeQueue
// Keys compare on their cached 16-byte normalized prefix first (two integer compares); only ties
// between longer keys read the key bytes (reference comparator semantics: CompareFunc.cc:70-91).
bool MergeQueue::less(const Segment* a, const Segment* b) {
  ++compares_;
  bool full = false;
  int c = keynorm_compare(a->norm, b->norm, &full);
  if (full) {
    const RecordView& x = a->cur();
    const RecordView& y = b->cur();
    c = key_compare(kind_, x.key, x.klen, y.key, y.klen);
  }
  if (c != 0) return c < 0;
  return a->index < b->index;
}

void MergeQueue::normalize(Segment* s) {
  const RecordView& r = s->cur();
  s->norm = key_normalize(kind_, r.key, r.klen);
}

void MergeQueue::up(size_t i) {
  while (i > 0) {
    size_t p = (i - 1) / 2;
    if (!less(heap_[i].get(), heap_[p].get())) break;
    std::swap(heap_[i], heap_[p]);
    i = p;
  }
}

void MergeQueue::down(size_t i) {
  const size_t n = heap_.size();
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < n && less(heap_[l].get(), heap_[m].get())) m = l;
    if (r < n && less(heap_[r].get(), heap_[m].get())) m = r;
    if (m == i) return;
    std::swap(heap_[i], heap_[m]);
    i = m;
  }
}

void MergeQueue::insert(std::unique_ptr<Segment> s) {
  if (!s->next()) return;  // empty segment
  normalize(s.get());
  heap_.push_back(std::move(s));
  up(heap_.size() - 1);
}

bool MergeQueue::next() {
  if (pending_advance_ && !heap_.empty()) {
    if (heap_[0]->next()) {
      normalize(heap_[0].get());
      down(0);
    } else {
      std::swap(heap_[0], heap_.back());
      heap_.pop_back();
      if (!heap_.empty()) down(0);
    }
  }
  pending_advance_ = false;
  if (heap_.empty()) {
    min_ = nullptr;
    return false;
  }
  min_ = heap_[0].get();
  pending_advance_ = true;
  return true;
}

// ---------------------------------------------------------------------------- KVWriter
bool KVWriter::fill(uint8_t* buf, int64_t cap, int64_t* len) {
  int64_t w = 0;
  for (;;) {
    if (!pending_) {
      if (drained_ || !q_->next()) {
        drained_ = true;
        break;
      }
      pending_ = true;
    }
    const RecordView& r = q_->cur();
    const int64_t need = ifile_record_size(r.klen, r.vlen);
    if (need > cap) throw UdaError("record larger than the delivery buffer");
    if (w + need > cap) {
      *len = w;
      return false;
    }
    w += ifile_write(buf + w, r.key, r.klen, r.val, r.vlen);
    pending_ = false;
    ++records_;
    bytes_ += need;
  }
  if (w + kEofBytes > cap) {
    *len = w;
    return false;
  }
  buf[w] = 0xFF;
  buf[w + 1] = 0xFF;
  *len = w + kEofBytes;
  return true;
}

}  // namespace uda
