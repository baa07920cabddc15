// Native token data loader for fine-tuning (C++ runtime; SURVEY §7.2 data layer).
//
// torch.classes.mxllm.TokenLoader(tokens, seq_len, batch, rank, world, seed, pin)
//   * tokens: int32 [N] — the packed token stream (documents joined by EOS);
//     it is cut into N // (seq_len + 1) training sequences;
//   * sharding = DistributedSampler semantics: per epoch a seeded permutation
//     (seed + epoch) of the sequences, padded to a multiple of world by
//     wrapping, rank r takes positions r, r + world, ...; every rank sees
//     disjoint sequences and the same number of batches;
//   * a background thread assembles (ids, labels) int64 [batch, seq_len]
//     batches into (pinned, when a GPU is present) host tensors, keeping a
//     bounded queue of `depth` batches ahead so the H2D copy is a single
//     non_blocking transfer and the GPU never waits on Python collation;
//   * state() / restore(epoch, cursor) make resume exact (checkpointing).
// pack(docs, eos): joins a list of int32 token tensors with EOS separators.
#include <torch/custom_class.h>
#include <torch/library.h>
#include <ATen/ATen.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <numeric>
#include <random>
#include <thread>

namespace {

class TokenLoader : public torch::CustomClassHolder {
 public:
  TokenLoader(at::Tensor tokens, int64_t seq_len, int64_t batch, int64_t rank, int64_t world, int64_t seed,
              bool pin, int64_t depth)
      : seq_(seq_len), batch_(batch), rank_(rank), world_(world), seed_(seed), pin_(pin),
        depth_(std::max<int64_t>(1, depth)) {
    TORCH_CHECK(tokens.dim() == 1 && tokens.scalar_type() == at::kInt, "tokens must be int32 [N]");
    TORCH_CHECK(seq_len > 0 && batch > 0 && world > 0 && rank >= 0 && rank < world, "bad loader geometry");
    tokens_ = tokens.contiguous().cpu();
    nseq_ = tokens_.numel() / (seq_ + 1);
    TORCH_CHECK(nseq_ > 0, "token stream shorter than one sequence");
    per_rank_ = (nseq_ + world_ - 1) / world_;
    nbatch_ = std::max<int64_t>(1, per_rank_ / batch_);
    start_epoch(0, 0);
    worker_ = std::thread([this] { run(); });
  }

  ~TokenLoader() override { shutdown(); }

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

  // returns (ids, labels, epoch, index_in_epoch)
  std::tuple<at::Tensor, at::Tensor, int64_t, int64_t> next() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return !q_.empty() || stop_; });
    TORCH_CHECK(!q_.empty(), "TokenLoader stopped");
    auto item = q_.front();
    q_.pop_front();
    consumed_epoch_ = std::get<2>(item);
    consumed_cursor_ = std::get<3>(item) + 1;
    cv_.notify_all();
    return item;
  }

  // (epoch, cursor) of the next batch the consumer will receive
  std::tuple<int64_t, int64_t> state() {
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
  void start_epoch(int64_t epoch, int64_t cursor) {
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
    const int32_t* tok = tokens_.data_ptr<int32_t>();
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
      auto opts = at::TensorOptions().dtype(at::kLong).pinned_memory(pin_);
      at::Tensor ids = at::empty({batch_, seq_}, opts);
      at::Tensor lab = at::empty({batch_, seq_}, opts);
      int64_t* ip = ids.data_ptr<int64_t>();
      int64_t* lp = lab.data_ptr<int64_t>();
      for (int64_t b = 0; b < batch_; ++b) {
        const int32_t* s = tok + idx[b] * (seq_ + 1);
        for (int64_t t = 0; t < seq_; ++t) {
          ip[b * seq_ + t] = s[t];
          lp[b * seq_ + t] = s[t + 1];
        }
      }
      std::lock_guard<std::mutex> g(mu_);
      if (gen != generation_) continue;  // restore() happened meanwhile: drop stale batch
      q_.emplace_back(ids, lab, e, c);
      cv_.notify_all();
    }
  }

  at::Tensor tokens_;
  int64_t seq_, batch_, rank_, world_, seed_;
  bool pin_;
  int64_t depth_;
  int64_t nseq_ = 0, per_rank_ = 0, nbatch_ = 0;
  int64_t epoch_ = 0, cursor_ = 0, generation_ = 0;
  int64_t consumed_epoch_ = 0, consumed_cursor_ = 0;
  std::vector<int64_t> perm_, mine_;
  std::deque<std::tuple<at::Tensor, at::Tensor, int64_t, int64_t>> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  std::thread worker_;
};

at::Tensor pack_documents(const std::vector<at::Tensor>& docs, int64_t eos) {
  int64_t n = 0;
  for (auto& d : docs) n += d.numel() + 1;
  auto out = at::empty({n}, at::TensorOptions().dtype(at::kInt));
  int32_t* o = out.data_ptr<int32_t>();
  for (auto& d0 : docs) {
    auto d = d0.to(at::kInt).contiguous().cpu();
    const int32_t* p = d.data_ptr<int32_t>();
    std::copy(p, p + d.numel(), o);
    o += d.numel();
    *o++ = (int32_t)eos;
  }
  return out;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(mxllm, m) {
  m.class_<TokenLoader>("TokenLoader")
      .def(torch::init<at::Tensor, int64_t, int64_t, int64_t, int64_t, int64_t, bool, int64_t>())
      .def("next", &TokenLoader::next)
      .def("state", &TokenLoader::state)
      .def("restore", &TokenLoader::restore)
      .def("batches_per_epoch", &TokenLoader::batches_per_epoch)
      .def("num_sequences", &TokenLoader::num_sequences)
      .def("shutdown", &TokenLoader::shutdown);
  m.def("pack_documents(Tensor[] docs, int eos) -> Tensor", &pack_documents);
}
