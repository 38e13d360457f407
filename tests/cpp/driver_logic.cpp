// Host-only check of the SteppingDriver's pull logic (reference SteppingDriver.cpp:102-366)
// through the ISteppingDriver ABI: the nodes here are plain host-memory Sources / Filters /
// Sinks written against <gpusdrpipeline/Factories.h>, so this runs without a GPU (CPU suite,
// tests/test_driver_logic.py). The device chain is covered by abi_kats.cpp on the GPU box.
//
// Cases: a linear chain with small preferred sizes (many steps, partial consumption, a FIR-like
// count rule that retains history), output-size alignment, fan-out of one source port to two
// sinks (copy through getOutputCopier), a two-input sink fed by two chains, the one-upstream-per-
// sink-port rule, node naming/iteration, and a source that stops producing. Composite graphs
// (FilterDriver.cpp, FilterDriverFactory.cpp, PortRemapping*.cpp, ReadByteCountMonitor.cpp): an
// inner graph behind a FilterDriver driven by an outer SteppingDriver, the same graph built from a
// JSON "Component" definition (nodes from registered test factories), definition errors, and the
// read-byte-count monitor.
#include <gpusdrpipeline/Factories.h>

#include <cstdio>
#include <cstdlib>
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
  IBufferCopier* getOutputCopier(size_t) noexcept final { return noCopier ? nullptr : F()->getSysMemCopier(); }
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
  bool noCopier = false;

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
  // as MultiplyCcc (Multiply.cpp): the lagging port asks for the difference, the leading one for
  // nothing, so a free-running second input (a tone source) never runs ahead of the first
  size_t preferredInputBufferSize(size_t port) noexcept final {
    const size_t mine = mIn[port].pending.size(), other = mIn[1 - port].pending.size();
    return other > mine ? 4 * (other - mine) : (mine > other ? 0 : 40);
  }
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

void fanOutUnequalBuffers() {
  // fan-out to sinks that lend different amounts: readOutput writes only what the smallest lent
  // buffer can take (the first buffer is capped), so no step fails with OutOfRange
  Ref<CounterSource> src = new CounterSource(1000, 4);
  Ref<Collect> s1 = new Collect(256), s2 = new Collect(24);  // host buffers: 256 and 64 bytes
  Ref<ISteppingDriver> d = newDriver();
  THROW_IF_ERR(d->connect(src.get(), 0, s1.get(), 0));
  THROW_IF_ERR(d->connect(src.get(), 0, s2.get(), 0));
  run(d.get(), [&] { return s1->mIn.pending.size() + s2->mIn.pending.size(); });
  std::vector<int32_t> x(1000);
  std::iota(x.begin(), x.end(), 0);
  CHECK(s1->mIn.pending == x);
  CHECK(s2->mIn.pending == x);
  CHECK(src->reads == (1000 + 15) / 16);  // 64 bytes (the smaller lent buffer) per step
}

void fanOutErrorCancels() {
  // a failure after the checkouts (no output copier for a fan-out port) cancels every lent
  // buffer: no sink stays checked out, and the same sinks can lend again afterwards
  Ref<CounterSource> src = new CounterSource(100, 4);
  src->noCopier = true;
  Ref<Collect> s1 = new Collect(16), s2 = new Collect(16);
  Ref<ISteppingDriver> d = newDriver();
  THROW_IF_ERR(d->connect(src.get(), 0, s1.get(), 0));
  THROW_IF_ERR(d->connect(src.get(), 0, s2.get(), 0));
  CHECK(d->doFilter() == Status_InvalidState);
  CHECK(s1->mIn.lent == nullptr && s2->mIn.lent == nullptr);
  CHECK(s1->mIn.pending.empty() && s2->mIn.pending.empty());
  src->noCopier = false;
  run(d.get(), [&] { return s1->mIn.pending.size() + s2->mIn.pending.size(); });
  // the failed step's samples (one 64-byte buffer) were already read from the source and are
  // dropped with it; everything after arrives at both sinks
  std::vector<int32_t> rest(84);
  std::iota(rest.begin(), rest.end(), 16);
  CHECK(s1->mIn.pending == rest && s2->mIn.pending == rest);
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

// y[k] = sum_j (x[k D + j] + tone[k D + j]): the FilterDriver case's inner graph on the whole stream
std::vector<int32_t> compositeExpect(size_t n, int32_t toneStart, size_t T, size_t D) {
  std::vector<int32_t> x(n);
  for (size_t i = 0; i < n; ++i) x[i] = (int32_t)i + toneStart + (int32_t)i;
  return windowSums(x, T, D);
}

void filterDriverComposite() {
  // outer: Counter(0..2999) -> [FilterDriver: in.0 -> Adder.0 ; Counter(500..) -> Adder.1 ;
  //         Adder -> WindowSum(5, 2) -> out.0] -> Collect
  Ref<IFilterDriver> fd = unwrap(F()->getFilterDriverFactory()->createFilterDriver());
  Ref<CounterSource> tone = new CounterSource(500 + 4000, 4, 500);  // readOutput materialises what is left
  Ref<Adder> add = new Adder();
  Ref<WindowSum> w = new WindowSum(5, 2, 36);
  THROW_IF_ERR(fd->connect(tone.get(), 0, add.get(), 1));
  THROW_IF_ERR(fd->connect(add.get(), 0, w.get(), 0));
  Ref<IPortRemappingSink> in = unwrap(F()->getPortRemappingSinkFactory()->create());
  Ref<IPortRemappingSource> out = unwrap(F()->getPortRemappingSourceFactory()->create());
  in->addPortMapping(0, add.get(), 0);
  out->addPortMapping(0, w.get(), 0);
  fd->setDriverInput(in.get());
  fd->setDriverOutput(out.get());
  THROW_IF_ERR(fd->setupNode(add.get(), "adder"));

  Ref<CounterSource> src = new CounterSource(3000, 4);
  Ref<Collect> sink = new Collect(44);
  Ref<ISteppingDriver> d = newDriver();
  THROW_IF_ERR(d->connect(src.get(), 0, fd.get(), 0));
  THROW_IF_ERR(d->connect(fd.get(), 0, sink.get(), 0));
  run(d.get(), [&] { return sink->mIn.pending.size(); });
  CHECK(sink->mIn.pending == compositeExpect(3000, 500, 5, 2));

  // the inner graph seen from outside: its edges plus the delegate edges, and node attributes
  int edges = 0, inputAttr = 0;
  fd->iterateOverConnections(&edges, [](IDriver*, void* c, Source*, size_t, Sink*, size_t) noexcept {
    ++*static_cast<int*>(c);
  });
  CHECK(edges == 4);  // tone -> adder, adder -> window, fd -> in, out -> fd
  fd->iterateOverNodeAttributes(in.get(), &inputAttr, [](IDriver*, Node*, void* c, const char* k, const char* v) noexcept {
    if (std::string(k) == "inputNode" && std::string(v) == "true") ++*static_cast<int*>(c);
  });
  CHECK(inputAttr == 1);
  char name[16];
  bool found = false;
  CHECK(fd->getNodeName(add.get(), name, sizeof(name), &found) == 5 && found);

  // without delegates the FilterDriver reports InvalidState (FilterDriver.cpp:160-166)
  Ref<IFilterDriver> bare = unwrap(F()->getFilterDriverFactory()->createFilterDriver());
  CHECK(bare->requestBuffer(0, 16).status == Status_InvalidState);
  CHECK(bare->getOutputDataSize(0) == 0);
}

// Test node factories for the JSON component: parameters are read from the node's OWN definition
// ("T", "D", "start"), so a factory handed the whole component text would build the wrong node.
long jsonInt(const char* json, const char* key, long dflt) {
  const std::string k = std::string("\"") + key + "\":";
  const char* p = std::strstr(json, k.c_str());
  return p == nullptr ? dflt : std::strtol(p + k.size(), nullptr, 10);
}

struct TestFactory final : public INodeFactory {
  enum Kind { kCounter, kWindow, kAdder } kind;
  explicit TestFactory(Kind k) : kind(k) {}
  Result<Node> create(const char* json) noexcept final {
    if (std::strstr(json, "\"nodes\"") != nullptr) return ERR_RESULT(Status_InvalidArgument);  // whole component
    Node* n = nullptr;
    if (kind == kCounter) n = new CounterSource((int32_t)jsonInt(json, "total", 4500), 4, (int32_t)jsonInt(json, "start", 0));
    if (kind == kWindow) n = new WindowSum((size_t)jsonInt(json, "T", 1), (size_t)jsonInt(json, "D", 1), 36);
    if (kind == kAdder) n = new Adder();
    return makeRefResultNonNull<Node>(n);
  }
  REF_COUNTED(TestFactory);
};

void componentFromJson() {
  THROW_IF_ERR(registerDefaultNodeFactories());  // "Component" is reached by name
  THROW_IF_ERR(registerNodeFactory("TestCounter", new TestFactory(TestFactory::kCounter)));
  THROW_IF_ERR(registerNodeFactory("TestWindowSum", new TestFactory(TestFactory::kWindow)));
  THROW_IF_ERR(registerNodeFactory("TestAdder", new TestFactory(TestFactory::kAdder)));
  const char* def = R"({"nodes": {"tone": {"type": "TestCounter", "start": 500},
                                  "adder": {"type": "TestAdder"},
                                  "window": {"type": "TestWindowSum", "T": 5, "D": 2}},
                       "connections": [{"source": "tone", "sourcePort": 0, "sink": "adder", "sinkPort": 1},
                                       {"source": "adder", "target": "window"}],
                       "inputPorts": [{"exposedPort": 0, "mapped": {"node": "adder", "port": 0}}],
                       "outputPorts": [{"exposedPort": 0, "mapped": {"node": "window", "port": 0}}]})";
  Ref<Filter> comp = unwrap(createFilter("Component", def));
  Ref<CounterSource> src = new CounterSource(3000, 4);
  Ref<Collect> sink = new Collect(44);
  Ref<ISteppingDriver> d = newDriver();
  THROW_IF_ERR(d->connect(src.get(), 0, comp.get(), 0));
  THROW_IF_ERR(d->connect(comp.get(), 0, sink.get(), 0));
  run(d.get(), [&] { return sink->mIn.pending.size(); });
  CHECK(sink->mIn.pending == compositeExpect(3000, 500, 5, 2));
  // the nodes carry their ids as names in the component's driver
  IDriver* cd = static_cast<Node*>(comp.get())->asDriver();
  CHECK(cd != nullptr);
  int named = 0;
  if (cd != nullptr)
    cd->iterateOverNodes(&named, [](IDriver* drv, void* c, Node* n) noexcept {
      char nm[16];
      bool f = false;
      drv->getNodeName(n, nm, sizeof(nm), &f);
      if (f) ++*static_cast<int*>(c);
    });
  CHECK(named == 3);

  // "outputPort": "<id>" (the RF -> PCM form) maps exposed port 0
  const char* def2 = R"({"nodes": {"w": {"type": "TestWindowSum", "T": 2, "D": 1}},
                        "inputPorts": [{"exposedPort": 0, "mapped": {"node": "w", "port": 0}}],
                        "outputPort": "w"})";
  Ref<Filter> comp2 = unwrap(createFilter("Component", def2));
  Ref<CounterSource> src2 = new CounterSource(100, 4);
  Ref<Collect> sink2 = new Collect(64);
  Ref<ISteppingDriver> d2 = newDriver();
  THROW_IF_ERR(d2->connect(src2.get(), 0, comp2.get(), 0));
  THROW_IF_ERR(d2->connect(comp2.get(), 0, sink2.get(), 0));
  run(d2.get(), [&] { return sink2->mIn.pending.size(); });
  std::vector<int32_t> x(100);
  std::iota(x.begin(), x.end(), 0);
  CHECK(sink2->mIn.pending == windowSums(x, 2, 1));
}

void componentErrors() {
  IFilterDriverFactory* f = F()->getFilterDriverFactory();
  CHECK(f->create("{not json").status == Status_ParseError);
  CHECK(f->create(R"({"connections": []})").status == Status_ParseError);  // no "nodes"
  CHECK(f->create(R"({"nodes": {"a": {"T": 3}}})").status == Status_InvalidArgument);  // no type
  CHECK(f->create(R"({"nodes": {"a": {"type": "NoSuchNodeType"}}})").status == Status_NotFound);
  CHECK(f->create(R"({"nodes": {"a": {"type": "TestAdder"}},
                      "connections": [{"source": "a", "sink": "b"}]})")
            .status == Status_InvalidArgument);  // undefined sink
  CHECK(f->create(R"({"nodes": {"a": {"type": "TestAdder"}},
                      "inputPorts": [{"exposedPort": 0, "mapped": {"node": "zz", "port": 0}}]})")
            .status == Status_NotFound);
  CHECK(f->create(R"({"nodes": {"a": {"type": "TestCounter"}},
                      "inputPorts": [{"exposedPort": 0, "mapped": {"node": "a", "port": 0}}]})")
            .status == Status_InvalidArgument);  // a source is not a sink
}

void byteCountMonitor() {
  Ref<CounterSource> src = new CounterSource(1000, 4);
  Ref<WindowSum> w = new WindowSum(7, 3, 100);
  Ref<IReadByteCountMonitor> mon = unwrap(F()->getReadByteCountMonitorFactory()->create(w.get()));
  Ref<Collect> sink = new Collect(48);
  Ref<ISteppingDriver> d = newDriver();
  THROW_IF_ERR(d->connect(src.get(), 0, mon.get(), 0));
  THROW_IF_ERR(d->connect(mon.get(), 0, sink.get(), 0));
  run(d.get(), [&] { return sink->mIn.pending.size(); });
  std::vector<int32_t> x(1000);
  std::iota(x.begin(), x.end(), 0);
  CHECK(sink->mIn.pending == windowSums(x, 7, 3));
  CHECK(mon->getByteCountRead(0) == 4 * sink->mIn.pending.size());
  CHECK(mon->getByteCountRead(3) == 0);
  CHECK(F()->getReadByteCountMonitorFactory()->create(nullptr).status == Status_InvalidArgument);
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
  runCase("fan_out_unequal_buffers", fanOutUnequalBuffers);
  runCase("fan_out_error_cancels", fanOutErrorCancels);
  runCase("two_inputs", twoInputs);
  runCase("connect_rules_and_names", connectRulesAndNames);
  runCase("exhausted_source", exhaustedSource);
  runCase("filter_driver_composite", filterDriverComposite);
  runCase("component_from_json", componentFromJson);
  runCase("component_errors", componentErrors);
  runCase("byte_count_monitor", byteCountMonitor);
  printf("%s (%d failures)\n", gFailures == 0 ? "ALL PASS" : "FAILURES", gFailures);
  return gFailures == 0 ? 0 : 1;
}
