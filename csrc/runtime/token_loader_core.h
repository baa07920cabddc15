// Torch-free core of the native token loader (csrc/runtime/dataloader.cpp).
//
// Kept free of ATen so the threading / sharding logic can be built and run
// standalone under AddressSanitizer + UBSan and ThreadSanitizer
// (tests/native/test_loader_core.cpp, driven by tests/test_native_sanitizers.py;
// SURVEY §5.2).  The torch class instantiates it with at::Tensor buffers
// (pinned host memory); the sanitizer driver with std::vector<int64_t>.
//
// Semantics (DistributedSampler-like, reference src/distributed_inference.py:58,63):
//   * the token stream is cut into nseq = N / (seq + 1) sequences;
//   * epoch e: seeded permutation (seed, e) of the sequences, padded to a
//     multiple of world by wrapping; rank r takes positions r, r + world, ...;
//   * a worker thread keeps up to `depth` assembled batches queued;
//   * state() / restore(epoch, cursor) give exact resume.
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <numeric>
#include <random>
#include <stdexcept>
#include <thread>
#include <tuple>
#include <utility>
#include <vector>

namespace mxrt {

template <class Buf>
class LoaderCore {
 public:
  using AllocFn = std::function<Buf(int64_t n)>;      // n int64 elements
  using PtrFn = std::function<int64_t*(Buf&)>;
  struct Item {
    Buf ids, lab;
    int64_t epoch, index;
  };

  LoaderCore(const int32_t* tokens, int64_t n_tokens, int64_t seq_len, int64_t batch, int64_t rank, int64_t world,
             int64_t seed, int64_t depth, AllocFn alloc, PtrFn ptr)
      : tok_(tokens), seq_(seq_len), batch_(batch), rank_(rank), world_(world), seed_(seed),
        depth_(std::max<int64_t>(1, depth)), alloc_(std::move(alloc)), ptr_(std::move(ptr)) {
    if (seq_len <= 0 || batch <= 0 || world <= 0 || rank < 0 || rank >= world) throw std::invalid_argument("bad loader geometry");
    nseq_ = n_tokens / (seq_ + 1);
    if (nseq_ <= 0) throw std::invalid_argument("token stream shorter than one sequence");
    per_rank_ = (nseq_ + world_ - 1) / world_;
    nbatch_ = std::max<int64_t>(1, per_rank_ / batch_);
    start_epoch(0, 0);
    worker_ = std::thread([this] { run(); });
  }

  ~LoaderCore() { shutdown(); }

  LoaderCore(const LoaderCore&) = delete;
  LoaderCore& operator=(const LoaderCore&) = delete;

  void shutdown() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
  }

  int64_t batches_per_epoch() const { return nbatch_; }
  int64_t num_sequences() const { return nseq_; }

  Item next() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return !q_.empty() || stop_; });
    if (q_.empty()) throw std::runtime_error("TokenLoader stopped");
    Item item = std::move(q_.front());
    q_.pop_front();
    consumed_epoch_ = item.epoch;
    consumed_cursor_ = item.index + 1;
    cv_.notify_all();
    return item;
  }

  // (epoch, cursor) of the next batch the consumer will receive
  std::pair<int64_t, int64_t> state() {
    std::lock_guard<std::mutex> g(mu_);
    if (consumed_cursor_ >= nbatch_) return {consumed_epoch_ + 1, 0};
    return {consumed_epoch_, consumed_cursor_};
  }

  void restore(int64_t epoch, int64_t cursor) {
    std::lock_guard<std::mutex> g(mu_);
    q_.clear();
    start_epoch(epoch, cursor);
    consumed_epoch_ = epoch;
    consumed_cursor_ = cursor;
    cv_.notify_all();
  }

 private:
  void start_epoch(int64_t epoch, int64_t cursor) {  // mu_ held (or constructor)
    epoch_ = epoch;
    cursor_ = cursor;
    perm_.resize(nseq_);
    std::iota(perm_.begin(), perm_.end(), 0);
    std::mt19937_64 rng((uint64_t)seed_ * 0x9E3779B97F4A7C15ull + (uint64_t)epoch);
    std::shuffle(perm_.begin(), perm_.end(), rng);
    const int64_t total = per_rank_ * world_;
    mine_.clear();
    for (int64_t i = rank_; i < total; i += world_) mine_.push_back(perm_[i % nseq_]);
    ++generation_;
  }

  void run() {
    while (true) {
      int64_t e, c, gen;
      std::vector<int64_t> idx;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || (int64_t)q_.size() < depth_; });
        if (stop_) return;
        if (cursor_ >= nbatch_) start_epoch(epoch_ + 1, 0);
        e = epoch_;
        c = cursor_++;
        gen = generation_;
        idx.assign(mine_.begin() + c * batch_, mine_.begin() + (c + 1) * batch_);
      }
      Buf ids = alloc_(batch_ * seq_);
      Buf lab = alloc_(batch_ * seq_);
      int64_t* ip = ptr_(ids);
      int64_t* lp = ptr_(lab);
      for (int64_t b = 0; b < batch_; ++b) {
        const int32_t* s = tok_ + idx[b] * (seq_ + 1);
        for (int64_t t = 0; t < seq_; ++t) {
          ip[b * seq_ + t] = s[t];
          lp[b * seq_ + t] = s[t + 1];
        }
      }
      std::lock_guard<std::mutex> g(mu_);
      if (gen != generation_) continue;  // restore() happened meanwhile: drop the stale batch
      q_.push_back(Item{std::move(ids), std::move(lab), e, c});
      cv_.notify_all();
    }
  }

  const int32_t* tok_;
  int64_t seq_, batch_, rank_, world_, seed_, depth_;
  AllocFn alloc_;
  PtrFn ptr_;
  int64_t nseq_ = 0, per_rank_ = 0, nbatch_ = 0;
  int64_t epoch_ = 0, cursor_ = 0, generation_ = 0;
  int64_t consumed_epoch_ = 0, consumed_cursor_ = 0;
  std::vector<int64_t> perm_, mine_;
  std::deque<Item> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  std::thread worker_;  // last member: started after everything it reads is constructed
};

}  // namespace mxrt
