// Standalone driver for mxrt::LoaderCore (csrc/runtime/token_loader_core.h),
// built by tests/test_native_sanitizers.py with -fsanitize=address,undefined
// and with -fsanitize=thread.  Exercises: sharding/coverage over epochs,
// label shift, exact resume, restore racing the producer thread, shutdown
// while the producer is blocked on a full queue, and destruction with
// batches still queued.  Exit code 0 = all checks passed.
#include <cstdio>
#include <set>
#include <vector>

#include "runtime/token_loader_core.h"

using Buf = std::vector<int64_t>;
using Core = mxrt::LoaderCore<Buf>;

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

static Core* make(const std::vector<int32_t>& toks, int64_t seq, int64_t batch, int64_t rank, int64_t world,
                  int64_t depth) {
  return new Core(toks.data(), (int64_t)toks.size(), seq, batch, rank, world, /*seed=*/7, depth,
                  [](int64_t n) { return Buf((size_t)n); }, [](Buf& b) { return b.data(); });
}

int main() {
  const int64_t seq = 16, batch = 3, world = 3;
  std::vector<int32_t> toks(40 * (seq + 1) + 5);
  for (size_t i = 0; i < toks.size(); ++i) toks[i] = (int32_t)i;  // token == position: sequences identifiable

  // 1. sharding: per epoch the ranks' first tokens are disjoint, labels = ids shifted by one
  for (int epoch = 0; epoch < 2; ++epoch) {
    std::set<int64_t> seen;
    int64_t total = 0;
    for (int64_t r = 0; r < world; ++r) {
      Core* c = make(toks, seq, batch, r, world, 2);
      if (epoch) c->restore(epoch, 0);
      for (int64_t b = 0; b < c->batches_per_epoch(); ++b) {
        auto it = c->next();
        CHECK(it.epoch == epoch && it.index == b);
        for (int64_t i = 0; i < batch; ++i) {
          const int64_t first = it.ids[i * seq];
          CHECK(first % (seq + 1) == 0);
          for (int64_t t = 0; t < seq; ++t) CHECK(it.lab[i * seq + t] == it.ids[i * seq + t] + 1);
          seen.insert(first);
          ++total;
        }
      }
      delete c;
    }
    CHECK((int64_t)seen.size() == total);  // 40 sequences, 3 ranks x 4 batches x 3 = 36 draws, all distinct
  }

  // 2. exact resume: state after k batches, restore in a fresh loader, identical stream
  {
    Core* a = make(toks, seq, batch, 1, world, 3);
    for (int i = 0; i < 2; ++i) a->next();
    auto st = a->state();
    std::vector<Buf> ref;
    for (int i = 0; i < 5; ++i) ref.push_back(a->next().ids);  // crosses an epoch boundary
    Core* b = make(toks, seq, batch, 1, world, 1);
    b->restore(st.first, st.second);
    for (int i = 0; i < 5; ++i) CHECK(b->next().ids == ref[(size_t)i]);
    delete a;
    delete b;
  }

  // 3. restore racing the producer (many times), consumer keeps reading
  {
    Core* c = make(toks, seq, batch, 0, 1, 4);
    for (int i = 0; i < 200; ++i) {
      c->restore(i % 3, i % 5);
      auto it = c->next();
      CHECK(it.epoch == i % 3 && it.index == i % 5);
    }
    delete c;
  }

  // 4. shutdown while the producer waits on a full queue; next() after shutdown drains then throws
  {
    Core* c = make(toks, seq, batch, 0, 1, 2);
    c->next();
    c->shutdown();
    bool threw = false;
    try {
      for (int i = 0; i < 10; ++i) c->next();
    } catch (const std::runtime_error&) {
      threw = true;
    }
    CHECK(threw);
    delete c;
  }

  // 5. destroy with batches queued (worker joined by the destructor)
  for (int i = 0; i < 20; ++i) delete make(toks, seq, batch, i % world, world, 8);

  std::printf("loader core: %s (%d failures)\n", failures ? "FAIL" : "ok", failures);
  return failures ? 1 : 0;
}
