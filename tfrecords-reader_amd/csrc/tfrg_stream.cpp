// tfrg_stream.cpp — double-buffered host -> HBM decode stream (include/tfrg.h, tfrg_stream_*).
//
// Replaces the reference's per-record ThreadPool read+decode (reader.py:212-247) and per-file
// process pool (indexer.py:121-134) for whole-dataset reads: two slots, each with a pinned host
// staging buffer (hipHostMalloc), a device input buffer and its own decode context + stream. A
// worker thread stages a submitted batch (its file images copied into pinned memory by a few copy
// threads, every piece indexed with the native framing walk), enqueues the H2D copies and the decode
// on the slot's stream, and moves on to the next batch; so the staging of batch k+1 and its H2D
// overlap the decode of batch k and the caller's consumption of batch k-1. Each slot has its own
// worker thread; after the decode it copies the result columns into the slot's pinned result
// buffers (exact sizes from the decode's summary), so the consumer reads them in place.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tfrg.h"

// tfrg_host.cpp: the framing walk of tfrg_index_buffer writing split, shifted columns
extern "C" int64_t tfrg_index_split(const uint8_t* file, uint64_t size, uint64_t base, uint64_t* starts,
                                    uint64_t* ends, int64_t cap);

namespace tfrg {
void set_error(const std::string& s);
}
using tfrg::set_error;

namespace {

// a piece of a batch: file bytes [off, off + size) (read with pread: no page faults of an mmap),
// or host memory (an inflated compressed file)
struct Piece {
  const uint8_t* ptr;
  std::string path;
  uint64_t off, size;
};

struct Job {
  int slot;
  uint32_t flags;
  std::vector<Piece> pieces;
};

// slot states
constexpr int kFree = 0, kStaging = 1, kReady = 2, kFailed = 3;

}  // namespace

// pinned host copy of one slot's result columns
struct PinnedCols {
  void* p = nullptr;
  size_t cap = 0;
  tfrg_columns cols{};
  tfrg_info info{};
};

// pinned allocation flags (TFRG_PINNED_IN / TFRG_PINNED_OUT override, for measurements)
static unsigned pinned_flags(const char* env, unsigned dflt) {
  const char* v = getenv(env);
  return v ? (unsigned)strtoul(v, nullptr, 0) : dflt;
}

struct tfrg_stream {
  int device = 0;
  unsigned in_flags = 0, out_flags = 0;
  uint64_t cap = 0;       // staging bytes per slot
  uint64_t max_rec = 0;   // records per slot (a framed record is >= 16 bytes)
  int copy_threads = 4;
  tfrg_ctx* ctx[2] = {nullptr, nullptr};
  uint8_t* h_buf[2] = {nullptr, nullptr};
  uint64_t* h_se[2] = {nullptr, nullptr};  // pinned [start..., end...]
  uint8_t* d_buf[2] = {nullptr, nullptr};
  uint64_t* d_se[2] = {nullptr, nullptr};
  hipStream_t stream[2] = {nullptr, nullptr};
  std::thread worker[2];
  std::mutex m;
  std::condition_variable cv;
  std::deque<Job> jobs[2];
  PinnedCols res[2];
  int state[2] = {kFree, kFree};
  int err[2] = {0, 0};
  std::string err_msg[2];
  uint64_t n_rec[2] = {0, 0}, n_bytes[2] = {0, 0};
  std::vector<uint64_t> piece_recs[2];
  double phase_ms[2][4] = {};  // per slot: read/copy, index, H2D + decode, D2H of the columns
  bool stop = false;
};

// the pieces copied back to back into dst by `threads` threads (8 MiB chunks); false on a read error
static bool parallel_copy(uint8_t* dst, const Job& j, int threads) {
  struct Chunk {
    uint8_t* d;
    const uint8_t* s;  // memory piece, or
    int fd;            // file piece
    uint64_t off, n;
  };
  std::vector<int> fds;
  std::vector<Chunk> chunks;
  uint64_t at = 0;
  bool ok = true;
  for (const Piece& p : j.pieces) {
    int fd = -1;
    if (!p.ptr) {
      fd = open(p.path.c_str(), O_RDONLY);
      if (fd < 0) {
        ok = false;
        break;
      }
      fds.push_back(fd);
    }
    for (uint64_t o = 0; o < p.size; o += (8u << 20)) {
      const uint64_t n = std::min<uint64_t>(8u << 20, p.size - o);
      chunks.push_back({dst + at + o, p.ptr ? p.ptr + o : nullptr, fd, p.off + o, n});
    }
    at += p.size;
  }
  std::vector<char> bad(chunks.size(), 0);
  auto run = [&](size_t c) {
    const Chunk& k = chunks[c];
    if (k.s) {
      memcpy(k.d, k.s, k.n);
      return;
    }
    uint64_t done = 0;
    while (done < k.n) {
      const ssize_t r = pread(k.fd, k.d + done, k.n - done, (off_t)(k.off + done));
      if (r <= 0) {
        bad[c] = 1;
        return;
      }
      done += (uint64_t)r;
    }
  };
  const int T = ok ? std::max(1, std::min<int>(threads, (int)chunks.size())) : 0;
  std::vector<std::thread> ts;
  for (int t = 1; t < T; ++t)
    ts.emplace_back([&, t] {
      for (size_t c = t; c < chunks.size(); c += T) run(c);
    });
  if (T)
    for (size_t c = 0; c < chunks.size(); c += T) run(c);
  for (auto& th : ts) th.join();
  for (int fd : fds) close(fd);
  for (char b : bad) ok &= !b;
  return ok;
}

static double ms_since(std::chrono::steady_clock::time_point& t) {
  const auto now = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(now - t).count();
  t = now;
  return ms;
}

static int stage_and_decode(tfrg_stream* s, const Job& j, double* ph) {
  const int k = j.slot;
  uint64_t total = 0;
  for (const Piece& p : j.pieces) total += p.size;
  if (total > s->cap) {
    set_error("batch larger than the stream's staging buffer");
    return TFRG_E_LIMIT;
  }
  // the slot's previous batch (H2D + decode) must be complete before its buffers are rewritten
  if (hipSetDevice(s->device) != hipSuccess || hipStreamSynchronize(s->stream[k]) != hipSuccess) {
    set_error("stream synchronize failed");
    return TFRG_E_HIP;
  }
  auto t = std::chrono::steady_clock::now();
  const bool copied = parallel_copy(s->h_buf[k], j, s->copy_threads);
  ph[0] = ms_since(t);
  if (!copied) {
    set_error("reading a TFRecord file piece failed");
    return TFRG_E_IO;
  }
  // framing index of every piece (bit-exact with indexer.pyx:212-252), pieces in parallel: a count
  // walk, then a second walk writing each piece's (start, end) columns, shifted to its offset in the
  // batch, straight into the pinned staging index (both walks touch 8 bytes per record)
  const size_t P = j.pieces.size();
  std::vector<uint64_t> base(P + 1, 0), cnt(P, 0), first(P + 1, 0);
  for (size_t i = 0; i < P; ++i) base[i + 1] = base[i] + j.pieces[i].size;
  const int T = std::max(1, std::min<int>(s->copy_threads, (int)P));
  auto run = [&](auto&& body) {
    std::vector<std::thread> ts;
    for (int q = 1; q < T; ++q) ts.emplace_back(body, q);
    body(0);
    for (auto& th : ts) th.join();
  };
  run([&](int q) {
    for (size_t i = q; i < P; i += T) {
      const int64_t c = tfrg_index_buffer(s->h_buf[k] + base[i], j.pieces[i].size, nullptr, 0);
      cnt[i] = c > 0 ? (uint64_t)c : 0u;
    }
  });
  for (size_t i = 0; i < P; ++i) first[i + 1] = first[i] + cnt[i];
  const uint64_t n = first[P];
  if (n > s->max_rec) {
    set_error("too many records for the stream's staging buffer");
    return TFRG_E_LIMIT;
  }
  uint64_t* st = s->h_se[k];
  run([&](int q) {
    for (size_t i = q; i < P; i += T)
      if (cnt[i])
        tfrg_index_split(s->h_buf[k] + base[i], j.pieces[i].size, base[i], st + first[i],
                         st + s->max_rec + first[i], (int64_t)cnt[i]);
  });
  s->piece_recs[k].assign(cnt.begin(), cnt.end());
  ph[1] = ms_since(t);
  memset(s->h_buf[k] + total, 0, 16);  // readable padding past the last record
  const uint64_t pad = (total + 15) & ~15ull;
  if (hipMemcpyAsync(s->d_buf[k], s->h_buf[k], pad + 16, hipMemcpyHostToDevice,
                     s->stream[k]) != hipSuccess ||
      (n && hipMemcpyAsync(s->d_se[k], st, n * 8, hipMemcpyHostToDevice, s->stream[k]) != hipSuccess) ||
      (n && hipMemcpyAsync(s->d_se[k] + s->max_rec, st + s->max_rec, n * 8, hipMemcpyHostToDevice, s->stream[k]) !=
                hipSuccess)) {
    set_error("H2D copy failed");
    return TFRG_E_HIP;
  }
  s->n_rec[k] = n;
  s->n_bytes[k] = total;
  if (total >= (1ull << 32)) {
    set_error("batch larger than 4 GiB");
    return TFRG_E_LIMIT;
  }
  const int rc = tfrg_decode_device(s->ctx[k], s->d_buf[k], total, s->d_se[k], s->d_se[k] + s->max_rec, (uint32_t)n,
                                    j.flags, s->stream[k]);
  if (!rc) {
    const hipError_t e = hipStreamSynchronize(s->stream[k]);
    if (e != hipSuccess) {
      set_error(std::string("decode stream synchronize: ") + hipGetErrorString(e));
      return TFRG_E_HIP;
    }
  }
  ph[2] = ms_since(t);
  return rc;
}

// copy the decoded columns of slot k into its pinned result buffers (sizes from the summary)
static int fetch_pinned(tfrg_stream* s, int k, uint32_t flags) {
  PinnedCols& pc = s->res[k];
  tfrg_info& info = pc.info;
  int rc = tfrg_result_info(s->ctx[k], &info);
  if (rc) return rc;
  const uint64_t n = info.n_records, S = info.n_slots;
  const bool mat = (flags & TFRG_FLAG_MATERIALIZE_BYTES) != 0;
  struct Part {
    void** dst;
    size_t bytes;
  };
  tfrg_columns& c = pc.cols;
  memset(&c, 0, sizeof(c));
  const uint64_t nb = info.kind_totals[TFRG_KIND_BYTES];
  Part parts[] = {
      {(void**)&c.status, n * 4},
      {(void**)&c.aux, info.n_errors ? n * 8 : 0},  // defined only for failing records
      {(void**)&c.verdict, n},
      {(void**)&c.order, S * n * 2},
      {(void**)&c.row_splits, S * (n + 1) * 4},
      {(void**)&c.slot_base, S * 8},
      {(void**)&c.i64, info.kind_totals[TFRG_KIND_INT64] * 8},
      {(void**)&c.f32, info.kind_totals[TFRG_KIND_FLOAT] * 4},
      {(void**)&c.bytes_len, nb * 4},
      {(void**)&c.bytes_off, mat ? 0 : nb * 4},  // (views only without the byte column)
      {(void**)&c.bytes_data, mat ? info.bytes_data_len : 0},
      {(void**)&c.bytes_offsets, mat ? (nb + 1) * 8 : 0},
  };
  size_t total = 0;
  for (const Part& p : parts) total += (p.bytes + 63) & ~(size_t)63;
  if (total > pc.cap) {
    // pinned allocations are slow (page pinning): grow geometrically so a stream settles at once
    const size_t want = std::max(total + total / 2, 2 * pc.cap) + 4096;
    if (pc.p) (void)hipHostFree(pc.p);
    pc.p = nullptr;
    pc.cap = 0;
    if (hipHostMalloc(&pc.p, want, s->out_flags) != hipSuccess) {
      set_error("pinned result allocation failed");
      return TFRG_E_NOMEM;
    }
    pc.cap = want;
  }
  size_t at = 0;
  for (const Part& p : parts) {
    *p.dst = p.bytes ? (uint8_t*)pc.p + at : nullptr;
    at += (p.bytes + 63) & ~(size_t)63;
  }
  return tfrg_result_fetch(s->ctx[k], &c);  // async D2H into pinned memory, synchronised
}

static void worker_main(tfrg_stream* s, int k) {
  (void)hipSetDevice(s->device);
  for (;;) {
    Job j;
    {
      std::unique_lock<std::mutex> lk(s->m);
      s->cv.wait(lk, [&] { return s->stop || !s->jobs[k].empty(); });
      if (s->stop && s->jobs[k].empty()) return;
      j = std::move(s->jobs[k].front());
      s->jobs[k].pop_front();
    }
    double ph[4] = {0, 0, 0, 0};
    int rc = stage_and_decode(s, j, ph);
    auto t = std::chrono::steady_clock::now();
    if (!rc) rc = fetch_pinned(s, k, j.flags);
    ph[3] = ms_since(t);
    {
      std::lock_guard<std::mutex> lk(s->m);
      s->err[k] = rc;
      if (rc) s->err_msg[k] = tfrg_last_error();
      for (int q = 0; q < 4; ++q) s->phase_ms[k][q] = ph[q];
      s->state[k] = rc ? kFailed : kReady;
    }
    s->cv.notify_all();
  }
}

extern "C" {

int tfrg_stream_create(int device, uint64_t batch_bytes, int copy_threads, tfrg_stream** out) {
  *out = nullptr;
  if (batch_bytes < 64 || batch_bytes >= (1ull << 32)) {
    set_error("batch_bytes must be in [64, 4 GiB)");
    return TFRG_E_ARG;
  }
  tfrg_stream* s = new tfrg_stream();
  s->device = device;
  s->cap = batch_bytes;
  s->max_rec = batch_bytes / 16 + 1;
  s->copy_threads = copy_threads > 0 ? copy_threads : 4;
  // input staging is written by the CPU and read by DMA; results are written by DMA and read by the CPU
  s->in_flags = pinned_flags("TFRG_PINNED_IN", hipHostMallocNonCoherent);
  s->out_flags = pinned_flags("TFRG_PINNED_OUT", hipHostMallocNonCoherent);
  int rc = 0;
  if (hipSetDevice(device) != hipSuccess) rc = TFRG_E_HIP;
  for (int k = 0; k < 2 && !rc; ++k) {
    rc = tfrg_ctx_create(device, &s->ctx[k]);
    if (rc) break;
    if (hipStreamCreateWithFlags(&s->stream[k], hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&s->h_buf[k], batch_bytes + 32, s->in_flags) != hipSuccess ||
        hipHostMalloc((void**)&s->h_se[k], 2 * s->max_rec * 8, s->in_flags) != hipSuccess ||
        hipMalloc((void**)&s->d_buf[k], batch_bytes + 32) != hipSuccess ||
        hipMalloc((void**)&s->d_se[k], 2 * s->max_rec * 8) != hipSuccess) {
      set_error("stream allocation failed (pinned host / device buffers)");
      rc = TFRG_E_NOMEM;
    }
  }
  if (rc) {
    tfrg_stream_destroy(s);
    return rc;
  }
  for (int k = 0; k < 2; ++k) s->worker[k] = std::thread(worker_main, s, k);
  *out = s;
  return 0;
}

int tfrg_stream_destroy(tfrg_stream* s) {
  if (!s) return 0;
  {
    std::lock_guard<std::mutex> lk(s->m);
    s->stop = true;
  }
  s->cv.notify_all();
  for (auto& w : s->worker)
    if (w.joinable()) w.join();
  (void)hipSetDevice(s->device);
  for (int k = 0; k < 2; ++k) {
    if (s->stream[k]) (void)hipStreamSynchronize(s->stream[k]);
    if (s->ctx[k]) tfrg_ctx_destroy(s->ctx[k]);
    if (s->h_buf[k]) (void)hipHostFree(s->h_buf[k]);
    if (s->h_se[k]) (void)hipHostFree(s->h_se[k]);
    if (s->d_buf[k]) (void)hipFree(s->d_buf[k]);
    if (s->d_se[k]) (void)hipFree(s->d_se[k]);
    if (s->stream[k]) (void)hipStreamDestroy(s->stream[k]);
    if (s->res[k].p) (void)hipHostFree(s->res[k].p);
  }
  delete s;
  return 0;
}

tfrg_ctx* tfrg_stream_ctx(tfrg_stream* s, int slot) { return s && (slot == 0 || slot == 1) ? s->ctx[slot] : nullptr; }

int tfrg_stream_submit(tfrg_stream* s, int slot, const uint8_t* const* pieces, const char* const* paths,
                       const uint64_t* offsets, const uint64_t* sizes, int n_pieces, uint32_t flags) {
  if (!s || (slot != 0 && slot != 1) || n_pieces < 0) return TFRG_E_ARG;
  Job j;
  j.slot = slot;
  j.flags = flags;
  for (int i = 0; i < n_pieces; ++i) {
    const bool file = paths && paths[i];
    j.pieces.push_back({file ? nullptr : pieces[i], file ? std::string(paths[i]) : std::string(),
                        offsets ? offsets[i] : 0, sizes[i]});
  }
  {
    std::unique_lock<std::mutex> lk(s->m);
    if (s->state[slot] != kFree) {  // staging, or a result / failure nobody has waited for yet
      set_error(s->state[slot] == kStaging ? "slot busy: wait for it first"
                                           : "slot holds an unclaimed result: tfrg_stream_wait it first");
      return TFRG_E_ARG;
    }
    s->state[slot] = kStaging;
    s->jobs[slot].push_back(std::move(j));
  }
  s->cv.notify_all();
  return 0;
}

int tfrg_stream_wait(tfrg_stream* s, int slot, uint64_t* n_records, uint64_t* nbytes, uint64_t* piece_records,
                     int cap, double* stage_ms) {
  if (!s || (slot != 0 && slot != 1)) return TFRG_E_ARG;
  std::unique_lock<std::mutex> lk(s->m);
  s->cv.wait(lk, [&] { return s->state[slot] != kStaging; });
  if (s->state[slot] == kFree) {
    set_error("nothing submitted to this slot");
    return TFRG_E_ARG;
  }
  if (s->state[slot] == kFailed) {
    s->state[slot] = kFree;
    set_error(s->err_msg[slot]);
    return s->err[slot];
  }
  s->state[slot] = kFree;
  if (n_records) *n_records = s->n_rec[slot];
  if (nbytes) *nbytes = s->n_bytes[slot];
  if (stage_ms)
    for (int q = 0; q < 4; ++q) stage_ms[q] = s->phase_ms[slot][q];
  const auto& pr = s->piece_recs[slot];
  for (int i = 0; i < cap && i < (int)pr.size(); ++i) piece_records[i] = pr[i];
  return 0;
}

const uint8_t* tfrg_stream_host_buffer(tfrg_stream* s, int slot) {
  return s && (slot == 0 || slot == 1) ? s->h_buf[slot] : nullptr;
}

int tfrg_stream_result(tfrg_stream* s, int slot, tfrg_info* info, tfrg_columns* host) {
  if (!s || (slot != 0 && slot != 1)) return TFRG_E_ARG;
  *info = s->res[slot].info;
  *host = s->res[slot].cols;
  return 0;
}

int tfrg_stream_host_ranges(tfrg_stream* s, int slot, const uint64_t** starts, const uint64_t** ends) {
  if (!s || (slot != 0 && slot != 1)) return TFRG_E_ARG;
  *starts = s->h_se[slot];
  *ends = s->h_se[slot] + s->max_rec;
  return 0;
}

}  // extern "C"
