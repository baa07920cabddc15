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

#include <memory>

#include "runtime/token_loader_core.h"

namespace {

// Torch front-end of mxrt::LoaderCore (token_loader_core.h): batches are
// (pinned) host int64 tensors, handed out without a copy.
class TokenLoader : public torch::CustomClassHolder {
 public:
  TokenLoader(at::Tensor tokens, int64_t seq_len, int64_t batch, int64_t rank, int64_t world, int64_t seed,
              bool pin, int64_t depth) {
    TORCH_CHECK(tokens.dim() == 1 && tokens.scalar_type() == at::kInt, "tokens must be int32 [N]");
    TORCH_CHECK(seq_len > 0 && batch > 0 && world > 0 && rank >= 0 && rank < world, "bad loader geometry");
    tokens_ = tokens.contiguous().cpu();
    TORCH_CHECK(tokens_.numel() / (seq_len + 1) > 0, "token stream shorter than one sequence");
    const auto opts = at::TensorOptions().dtype(at::kLong).pinned_memory(pin);
    core_ = std::make_unique<mxrt::LoaderCore<at::Tensor>>(
        tokens_.data_ptr<int32_t>(), tokens_.numel(), seq_len, batch, rank, world, seed, depth,
        [opts, batch, seq_len](int64_t) { return at::empty({batch, seq_len}, opts); },
        [](at::Tensor& t) { return t.data_ptr<int64_t>(); });
  }

  ~TokenLoader() override { shutdown(); }

  void shutdown() {
    if (core_) core_->shutdown();
  }

  int64_t batches_per_epoch() const { return core_->batches_per_epoch(); }
  int64_t num_sequences() const { return core_->num_sequences(); }

  // returns (ids, labels, epoch, index_in_epoch)
  std::tuple<at::Tensor, at::Tensor, int64_t, int64_t> next() {
    try {
      auto it = core_->next();
      return {it.ids, it.lab, it.epoch, it.index};
    } catch (const std::exception& e) {
      TORCH_CHECK(false, e.what());
    }
  }

  std::tuple<int64_t, int64_t> state() {
    auto s = core_->state();
    return {s.first, s.second};
  }

  void restore(int64_t epoch, int64_t cursor) { core_->restore(epoch, cursor); }

 private:
  at::Tensor tokens_;  // owns the stream the core reads
  std::unique_ptr<mxrt::LoaderCore<at::Tensor>> core_;
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
