// Host-only check of the SteppingDriver's pull logic (reference SteppingDriver.cpp:102-366)
// through the ISteppingDriver ABI: the nodes here are plain host-memory Sources / Filters /
// Sinks written against <gpusdrpipeline/Factories.h>, so this runs without a GPU (CPU suite,
// tests/test_driver_logic.py). The device chain is covered by abi_kats.cpp on the GPU box.
//
// Cases: a linear chain with small preferred sizes (many steps, partial consumption, a FIR-like
// count rule that retains history), output-size alignment, fan-out of one source port to two
// sinks (copy through getOutputCopier), a two-input sink fed by two chains, the one-upstream-per-
// sink-port rule, node naming/iteration, and a source that stops producing.
#include <gpusdrpipeline/Factories.h>

#include <cstdio>
#include <cstring>
#include <functional>
#include <numeric>
#include <string>
#include <vector>

namespace {

int gFailures = 0;
#define CHECK(cond__)                                                              \
  do {                                                                             \
    if (!(cond__)) {                                                               \
      fprintf(stderr, "CHECK failed: %s at %s:%d\n", #cond__, __FILE__, __LINE__); \
      ++gFailures;                                                                 \
    }                                                                              \
  } while (false)

IFactories* F() {
  static IFactories* f = getFactoriesSingleton().value;
  return f;
}

IBufferFactory* hostBuffers() {
  static Ref<IBufferFactory> bf = unwrap(F()->createBufferFactory(F()->getSysMemAllocator()));
  return bf.get();
}

// One input port: lends a fresh host buffer, appends what is committed.
struct HostPort {
  std::vector<int32_t> pending;
  Ref<IBuffer> lent;
  size_t requests = 0;
  size_t lastRequest = 0;

  Result<IBuffer> request(size_t bytes) noexcept {
    if (lent != nullptr) return ERR_RESULT(Status_InvalidState);  // one checkout at a time
    Result<IBuffer> r = hostBuffers()->createBuffer(bytes == 0 ? 4 : bytes);
    if (r.status != Status_Success) return r;
    lent = r.value;
    ++requests;
    lastRequest = bytes;
    return r;
  }
  Status commit(size_t bytes) noexcept {
    if (lent == nullptr) return Status_InvalidState;
    if (bytes % 4 != 0 || bytes > lent.get()->range()->capacity()) return Status_InvalidArgument;
    const int32_t* p = reinterpret_cast<const int32_t*>(lent.get()->base());
    pending.insert(pending.end(), p, p + bytes / 4);
    lent.reset();
    return Status_Success;
  }
};

// Writes as many of `values` as fit into `out` (int32 elements), returns the count.
size_t emit(IBuffer* out, const int32_t* values, size_t n) {
  const size_t fit = std::min(n, out->range()->remaining() / 4);
  std::memcpy(out->writePtr(), values, fit * 4);
  (void)out->range()->increaseEndOffset(fit * 4);
  return fit;
}

// 0, 1, 2, ... up to `total` values; `alignment` bytes of output granularity.
class CounterSource final : public Source {
 public:
  CounterSource(int32_t total, size_t alignment, int32_t start = 0) : mTotal(total), mNext(start), mAlign(alignment) {}
  size_t getOutputDataSize(size_t) noexcept final { return 4 * (size_t)(mTotal - mNext); }
  size_t getOutputSizeAlignment(size_t) noexcept final { return mAlign; }
  IBufferCopier* getOutputCopier(size_t) noexcept final { return F()->getSysMemCopier(); }
  Status readOutput(IBuffer** outs, size_t n) noexcept final {
    if (n != mPorts) return Status_InvalidArgument;
    ++reads;
    std::vector<int32_t> v((size_t)(mTotal - mNext));
    std::iota(v.begin(), v.end(), mNext);
    const size_t wrote = emit(outs[0], v.data(), v.size());
    for (size_t p = 1; p < n; ++p)
      if (emit(outs[p], v.data(), wrote) != wrote) return Status_OutOfRange;
    mNext += (int32_t)wrote;
    return Status_Success;
  }
  void setPorts(size_t n) { mPorts = n; }
  int reads = 0;

 private:
  const int32_t mTotal;
  int32_t mNext;
  const size_t mAlign;
  size_t mPorts = 1;
  REF_COUNTED(CounterSource);
};

// FIR-like filter over int32: y[k] = sum_{j<T} x[kD + j]; count rule of Fir.cpp:178-186,
// consumes k*D inputs (history retained), preferred input size `pref` bytes.
class WindowSum final : public Filter {
 public:
  WindowSum(size_t T, size_t D, size_t pref) : mT(T), mD(D), mPref(pref) {}
  Result<IBuffer> requestBuffer(size_t port, size_t bytes) noexcept final {
    if (port != 0) return ERR_RESULT(Status_OutOfRange);
    return mIn.request(bytes);
  }
  Status commitBuffer(size_t port, size_t bytes) noexcept final { return port == 0 ? mIn.commit(bytes) : Status_OutOfRange; }
  size_t preferredInputBufferSize(size_t) noexcept final { return mPref; }
  size_t getOutputDataSize(size_t) noexcept final { return 4 * count(); }
  size_t getOutputSizeAlignment(size_t) noexcept final { return 4; }
  IBufferCopier* getOutputCopier(size_t) noexcept final { return F()->getSysMemCopier(); }
  Status readOutput(IBuffer** outs, size_t n) noexcept final {
    if (n != 1) return Status_InvalidArgument;
    std::vector<int32_t> y(count());
    for (size_t k = 0; k < y.size(); ++k) {
      int64_t s = 0;
      for (size_t j = 0; j < mT; ++j) s += mIn.pending[k * mD + j];
      y[k] = (int32_t)s;
    }
    const size_t wrote = emit(outs[0], y.data(), y.size());
    mIn.pending.erase(mIn.pending.begin(), mIn.pending.begin() + (ptrdiff_t)(wrote * mD));
    return Status_Success;
  }
  HostPort mIn;

 private:
  size_t count() const { return mIn.pending.size() < mT ? 0 : (mIn.pending.size() - (mT - 1)) / mD; }
  const size_t mT, mD, mPref;
  REF_COUNTED(WindowSum);
};

// Two input ports; output = in0 + in1 element-wise over the common prefix.
class Adder final : public Filter {
 public:
  Result<IBuffer> requestBuffer(size_t port, size_t bytes) noexcept final {
    if (port > 1) return ERR_RESULT(Status_OutOfRange);
    return mIn[port].request(bytes);
  }
  Status commitBuffer(size_t port, size_t bytes) noexcept final { return port > 1 ? Status_OutOfRange : mIn[port].commit(bytes); }
  size_t preferredInputBufferSize(size_t) noexcept final { return 40; }
  size_t getOutputDataSize(size_t) noexcept final { return 4 * std::min(mIn[0].pending.size(), mIn[1].pending.size()); }
  size_t getOutputSizeAlignment(size_t) noexcept final { return 4; }
  IBufferCopier* getOutputCopier(size_t) noexcept final { return F()->getSysMemCopier(); }
  Status readOutput(IBuffer** outs, size_t n) noexcept final {
    const size_t m = std::min(mIn[0].pending.size(), mIn[1].pending.size());
    std::vector<int32_t> y(m);
    for (size_t i = 0; i < m; ++i) y[i] = mIn[0].pending[i] + mIn[1].pending[i];
    const size_t wrote = emit(outs[0], y.data(), m);
    for (auto& p : mIn) p.pending.erase(p.pending.begin(), p.pending.begin() + (ptrdiff_t)wrote);
    return Status_Success;
  }
  HostPort mIn[2];
  REF_COUNTED(Adder);
};

class Collect final : public Sink {
 public:
  explicit Collect(size_t pref) : mPref(pref) {}
  Result<IBuffer> requestBuffer(size_t port, size_t bytes) noexcept final {
    if (port != 0) return ERR_RESULT(Status_OutOfRange);
    return mIn.request(bytes);
  }
  Status commitBuffer(size_t port, size_t bytes) noexcept final { return port == 0 ? mIn.commit(bytes) : Status_OutOfRange; }
  size_t preferredInputBufferSize(size_t) noexcept final { return mPref; }
  HostPort mIn;

 private:
  const size_t mPref;
  REF_COUNTED(Collect);
};

Ref<ISteppingDriver> newDriver() { return unwrap(F()->getSteppingDriverFactory()->createSteppingDriver()); }

// Step until the tail stops growing (a few extra steps to be sure nothing is left behind).
void run(ISteppingDriver* d, const std::function<size_t()>& progress, int maxSteps = 100000) {
  size_t last = progress();
  int idle = 0;
  for (int i = 0; i < maxSteps && idle < 8; ++i) {
    THROW_IF_ERR(d->doFilter());
    const size_t now = progress();
    idle = now == last ? idle + 1 : 0;
    last = now;
  }
}

// the whole-stream result under the reference count rule floor((N - (T - 1)) / D) (Fir.cpp:178-186)
std::vector<int32_t> windowSums(const std::vector<int32_t>& x, size_t T, size_t D) {
  std::vector<int32_t> y;
  const size_t n = x.size() < T ? 0 : (x.size() - (T - 1)) / D;
  for (size_t k = 0; k < n; ++k) {
    int64_t s = 0;
    for (size_t j = 0; j < T; ++j) s += x[k * D + j];
    y.push_back((int32_t)s);
  }
  return y;
}

void linearChain() {
  // Counter(10 000) -> WindowSum(T=7, D=3, pref 100 B) -> WindowSum(T=5, D=2, pref 64 B) -> Collect(48 B)
  Ref<CounterSource> src = new CounterSource(10000, 4);
  Ref<WindowSum> a = new WindowSum(7, 3, 100);
  Ref<WindowSum> b = new WindowSum(5, 2, 64);
  Ref<Collect> sink = new Collect(48);
  Ref<ISteppingDriver> d = newDriver();
  // connect downstream-first: tails must still come out right (SteppingDriver.cpp:126-132)
  THROW_IF_ERR(d->connect(b.get(), 0, sink.get(), 0));
  THROW_IF_ERR(d->connect(a.get(), 0, b.get(), 0));
  THROW_IF_ERR(d->connect(src.get(), 0, a.get(), 0));
  run(d.get(), [&] { return sink->mIn.pending.size(); });
  std::vector<int32_t> x(10000);
  std::iota(x.begin(), x.end(), 0);
  const std::vector<int32_t> expect = windowSums(windowSums(x, 7, 3), 5, 2);
  CHECK(sink->mIn.pending == expect);
  CHECK(sink->mIn.requests > 50);  // 48-byte buffers: many steps
  // nothing left that could still produce output
  CHECK(a->getOutputDataSize(0) == 0 && b->getOutputDataSize(0) == 0 && src->getOutputDataSize(0) == 0);
}

void alignment() {
  // a 32-byte output alignment rounds the 20-byte preferred request up to 32 bytes
  Ref<CounterSource> src = new CounterSource(100, 32);
  Ref<Collect> sink = new Collect(20);
  Ref<ISteppingDriver> d = newDriver();
  THROW_IF_ERR(d->connect(src.get(), 0, sink.get(), 0));
  THROW_IF_ERR(d->doFilter());
  CHECK(sink->mIn.lastRequest == 32);
  run(d.get(), [&] { return sink->mIn.pending.size(); });
  CHECK(sink->mIn.pending.size() == 100 && sink->mIn.pending[99] == 99);
}

void fanOut() {
  // one source port feeding two sinks: the second gets a copy (getOutputCopier)
  Ref<CounterSource> src = new CounterSource(1000, 4);
  Ref<Collect> s1 = new Collect(64), s2 = new Collect(64);
  Ref<ISteppingDriver> d = newDriver();
  THROW_IF_ERR(d->connect(src.get(), 0, s1.get(), 0));
  THROW_IF_ERR(d->connect(src.get(), 0, s2.get(), 0));
  run(d.get(), [&] { return s1->mIn.pending.size() + s2->mIn.pending.size(); });
  std::vector<int32_t> x(1000);
  std::iota(x.begin(), x.end(), 0);
  CHECK(s1->mIn.pending == x);
  CHECK(s2->mIn.pending == x);
  CHECK(src->reads == (1000 + 15) / 16);  // one readOutput per step serves both sinks
}

void twoInputs() {
  // Counter(0..) -> WindowSum(3,1) -> Adder.0 ; Counter(1000..) -> Adder.1 ; Adder -> Collect
  Ref<CounterSource> c0 = new CounterSource(500, 4), c1 = new CounterSource(1500, 4, 1000);
  Ref<WindowSum> w = new WindowSum(3, 1, 24);
  Ref<Adder> add = new Adder();
  Ref<Collect> sink = new Collect(1 << 20);
  Ref<ISteppingDriver> d = newDriver();
  THROW_IF_ERR(d->connect(c0.get(), 0, w.get(), 0));
  THROW_IF_ERR(d->connect(w.get(), 0, add.get(), 0));
  THROW_IF_ERR(d->connect(c1.get(), 0, add.get(), 1));
  THROW_IF_ERR(d->connect(add.get(), 0, sink.get(), 0));
  run(d.get(), [&] { return sink->mIn.pending.size(); });
  std::vector<int32_t> x(500);
  std::iota(x.begin(), x.end(), 0);
  const std::vector<int32_t> ws = windowSums(x, 3, 1);
  CHECK(sink->mIn.pending.size() == ws.size());
  bool ok = true;
  for (size_t i = 0; i < ws.size() && i < sink->mIn.pending.size(); ++i) ok &= sink->mIn.pending[i] == ws[i] + 1000 + (int32_t)i;
  CHECK(ok);
}

void connectRulesAndNames() {
  Ref<CounterSource> c0 = new CounterSource(10, 4), c1 = new CounterSource(10, 4);
  Ref<Collect> sink = new Collect(64);
  Ref<ISteppingDriver> d = newDriver();
  THROW_IF_ERR(d->connect(c0.get(), 0, sink.get(), 0));
  CHECK(d->connect(c1.get(), 0, sink.get(), 0) == Status_InvalidState);  // SteppingDriver.cpp:418-442
  CHECK(d->connect(nullptr, 0, sink.get(), 0) == Status_InvalidArgument);
  THROW_IF_ERR(d->setupNode(c0.get(), "counter"));
  THROW_IF_ERR(d->setupNode(sink.get(), "collector"));
  char name[32];
  bool found = false;
  CHECK(d->getNodeName(c0.get(), name, sizeof(name), &found) == 7 && found && std::string(name) == "counter");
  CHECK(d->getNodeName(c1.get(), name, sizeof(name), &found) == 0 && !found && name[0] == 0);
  char small[4];
  CHECK(d->getNodeName(sink.get(), small, sizeof(small), &found) == 9 && found && std::memcmp(small, "coll", 4) == 0);
  int nodes = 0, edges = 0;
  d->iterateOverNodes(&nodes, [](IDriver*, void* c, Node*) noexcept { ++*static_cast<int*>(c); });
  d->iterateOverConnections(&edges, [](IDriver*, void* c, Source*, size_t, Sink*, size_t) noexcept {
    ++*static_cast<int*>(c);
  });
  CHECK(nodes == 2 && edges == 1);
  CHECK(static_cast<Node*>(d.get())->asDriver() != nullptr);
}

void exhaustedSource() {
  // the source runs dry: steps after that are no-ops, not errors
  Ref<CounterSource> src = new CounterSource(5, 4);
  Ref<WindowSum> w = new WindowSum(3, 1, 1024);
  Ref<Collect> sink = new Collect(1024);
  Ref<ISteppingDriver> d = newDriver();
  THROW_IF_ERR(d->connect(src.get(), 0, w.get(), 0));
  THROW_IF_ERR(d->connect(w.get(), 0, sink.get(), 0));
  for (int i = 0; i < 5; ++i) THROW_IF_ERR(d->doFilter());
  CHECK((sink->mIn.pending == std::vector<int32_t>{3, 6, 9}));
}

void runCase(const char* name, void (*fn)()) {
  const int before = gFailures;
  try {
    fn();
  } catch (const std::exception& e) {
    fprintf(stderr, "%s threw: %s\n", name, e.what());
    ++gFailures;
  }
  printf("%-26s %s\n", name, gFailures == before ? "ok" : "FAILED");
}

}  // namespace

int main() {
  runCase("linear_chain", linearChain);
  runCase("alignment", alignment);
  runCase("fan_out", fanOut);
  runCase("two_inputs", twoInputs);
  runCase("connect_rules_and_names", connectRulesAndNames);
  runCase("exhausted_source", exhaustedSource);
  printf("%s (%d failures)\n", gFailures == 0 ? "ALL PASS" : "FAILURES", gFailures);
  return gFailures == 0 ? 0 : 1;
}
