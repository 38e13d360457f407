// Drop-in check of the gpusdrpipeline C++ ABI: the reference's known-answer tests
// (tests/FirTests.cpp:8-221, tests/CosineSourceTests.cpp:8-56) re-expressed as plain C++ against
// <gpusdrpipeline/Factories.h>, plus the JSON node registry and a chunked
// Int8ToFloat -> Fir -> QuadAmDemod chain driven through requestBuffer/commitBuffer/readOutput.
//
// Build: tests/cpp/Makefile. Run on a GPU box: tests/cpp/_build/abi_kats (exit 0 = all pass).
#include <gpusdrpipeline/Factories.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

namespace {

int gFailures = 0;

#define CHECK(cond__)                                                      \
  do {                                                                     \
    if (!(cond__)) {                                                       \
      fprintf(stderr, "CHECK failed: %s at %s:%d\n", #cond__, __FILE__, __LINE__); \
      ++gFailures;                                                         \
    }                                                                      \
  } while (false)

struct Cf {
  float re, im;
};

ConstRef<IFactories> F() {
  static ConstRef<IFactories> f = unwrap(getFactoriesSingleton());
  return f;
}

std::vector<uint8_t> toHost(IBuffer* b, ICudaCommandQueue* q) {
  ConstRef<IBufferCopier> d2h = unwrap(F()->getCudaBufferCopierFactory()->createBufferCopier(q, hipMemcpyDeviceToHost));
  std::vector<uint8_t> host(b->range()->used());
  THROW_IF_ERR(d2h->copy(host.data(), b->readPtr(), host.size()));
  if (hipStreamSynchronize(q->cudaStream()) != hipSuccess) throw std::runtime_error("sync");
  return host;
}

void push(Sink* sink, const void* host, size_t bytes, ICudaCommandQueue* q) {
  ConstRef<IBufferCopier> h2d = unwrap(F()->getCudaBufferCopierFactory()->createBufferCopier(q, hipMemcpyHostToDevice));
  ConstRef<IBuffer> in = unwrap(sink->requestBuffer(0, bytes));
  THROW_IF_ERR(h2d->copy(in->writePtr(), host, bytes));
  THROW_IF_ERR(sink->commitBuffer(0, bytes));
}

// FirTests.cpp:8-94 - two commits (3 + 2 samples), decimation 2, oversized output buffer.
void firTwoCommits(Filter* fir, ICudaCommandQueue* q) {
  const Cf a[] = {{0.1f, 0.2f}, {0.3f, 0.4f}, {0.5f, 0.6f}};
  const Cf b[] = {{0.7f, 0.8f}, {0.9f, 0.9f}};
  push(fir, a, sizeof(a), q);
  push(fir, b, sizeof(b), q);
  ConstRef<IAllocator> alloc = unwrap(F()->getCudaAllocatorFactory()->createCudaAllocator(q, 32, false));
  ConstRef<IBufferFactory> bf = unwrap(F()->createBufferFactory(alloc));
  const size_t outSize = 2 * fir->getOutputDataSize(0);
  CHECK(outSize == 2 * 2 * sizeof(Cf));
  ConstRef<IBuffer> out = unwrap(bf->createBuffer(outSize));
  CHECK(out->range()->used() == 0);
  IBuffer* outs[] = {out.get()};
  THROW_IF_ERR(fir->readOutput(outs, 1));
  CHECK(out->range()->used() == 2 * sizeof(Cf));
  std::vector<uint8_t> h = toHost(out, q);
  const Cf* y = reinterpret_cast<const Cf*>(h.data());
  const Cf expect[] = {{0.35f, 0.5f}, {0.95f, 1.1f}};
  for (int i = 0; i < 2; ++i) {
    CHECK(std::fabs(y[i].re - expect[i].re) < 1e-3f);
    CHECK(std::fabs(y[i].im - expect[i].im) < 1e-3f);
  }
}

// FirTests.cpp:96-221 - first read fits 1 output, second read 2: no input may be skipped.
void firPartialReads(ICudaCommandQueue* q) {
  const float taps[] = {0.5f, 1.0f, 0.25f};
  ConstRef<Filter> fir =
      unwrap(F()->getFirFactory()->createFir(SampleType_Float, SampleType_FloatComplex, 2, taps, 3, q));
  const Cf x[] = {{0.1f, 0.2f}, {0.3f, 0.4f}, {0.5f, 0.6f}, {0.7f, 0.8f},
                  {0.1f, 0.2f}, {0.3f, 0.4f}, {0.5f, 0.6f}, {0.7f, 0.8f}};
  push(fir.get(), x, sizeof(x), q);
  ConstRef<IAllocator> alloc =
      unwrap(F()->getCudaAllocatorFactory()->createCudaAllocator(q, fir->getOutputSizeAlignment(0), false));
  ConstRef<IBufferFactory> bf = unwrap(F()->createBufferFactory(alloc));
  ConstRef<IBuffer> raw1 = unwrap(bf->createBuffer(sizeof(Cf)));
  ConstRef<IBuffer> raw2 = unwrap(bf->createBuffer(2 * sizeof(Cf)));
  // the allocation is rounded up to the alignment, so slice to the exact sizes
  ConstRef<IBuffer> out1 = unwrap(F()->getBufferSliceFactory()->slice(raw1, 0, sizeof(Cf)));
  ConstRef<IBuffer> out2 = unwrap(F()->getBufferSliceFactory()->slice(raw2, 0, 2 * sizeof(Cf)));
  out1->range()->clearRange();
  out2->range()->clearRange();
  IBuffer* o1[] = {out1.get()};
  IBuffer* o2[] = {out2.get()};
  THROW_IF_ERR(fir->readOutput(o1, 1));
  THROW_IF_ERR(fir->readOutput(o2, 1));
  CHECK(out1->range()->used() == sizeof(Cf));
  CHECK(out2->range()->used() == 2 * sizeof(Cf));
  std::vector<uint8_t> h1 = toHost(out1, q), h2 = toHost(out2, q);
  const Cf* y1 = reinterpret_cast<const Cf*>(h1.data());
  const Cf* y2 = reinterpret_cast<const Cf*>(h2.data());
  CHECK(std::fabs(y1[0].re - 0.475f) < 1e-3f && std::fabs(y1[0].im - 0.65f) < 1e-3f);
  CHECK(std::fabs(y2[0].re - 0.975f) < 1e-3f && std::fabs(y2[0].im - 1.15f) < 1e-3f);
  CHECK(std::fabs(y2[1].re - 0.475f) < 1e-3f && std::fabs(y2[1].im - 0.65f) < 1e-3f);
}

// CosineSourceTests.cpp:8-56 - fs = 100, f = 1, 101 samples within 1e-4 of cos/sin.
void cosineSource(ICudaCommandQueue* q) {
  ConstRef<Source> src =
      unwrap(F()->getCosineSourceFactory()->createCosineSource(SampleType_FloatComplex, 100.0f, 1.0f, q));
  ConstRef<IAllocator> alloc = unwrap(F()->getCudaAllocatorFactory()->createCudaAllocator(q, 32, false));
  ConstRef<IBufferFactory> bf = unwrap(F()->createBufferFactory(alloc));
  ConstRef<IBuffer> out = unwrap(bf->createBuffer(101 * sizeof(Cf)));
  IBuffer* outs[] = {out.get()};
  THROW_IF_ERR(src->readOutput(outs, 1));
  CHECK(out->range()->used() == 104 * sizeof(Cf));  // fills the 32-byte-rounded capacity
  std::vector<uint8_t> h = toHost(out, q);
  const Cf* v = reinterpret_cast<const Cf*>(h.data());
  for (int i = 0; i <= 100; ++i) {
    const float theta = static_cast<float>(i) * 1.0f / 100.0f * static_cast<float>(M_PI) * 2.0f;
    CHECK(std::fabs(v[i].re - std::cos(theta)) < 1e-4f);
    CHECK(std::fabs(v[i].im - std::sin(theta)) < 1e-4f);
  }
}

// Node registry + named queue + JSON parameters (FilterFactories.cpp:27-150, FirFactory.h:28-53).
void jsonRegistry() {
  THROW_IF_ERR(registerDefaultNodeFactories());
  CHECK(hasNodeFactory("Fir") && hasNodeFactory("QuadDemod") && hasNodeFactory("Int8ToFloat"));
  THROW_IF_ERR(F()->getCommandQueueFactory()->create("kat", R"({"queueType": "hip", "cudaDevice": 0})"));
  ConstRef<ICudaCommandQueue> q = unwrap(F()->getCommandQueueFactory()->getCudaCommandQueue("kat"));
  ConstRef<Filter> fir = unwrap(createFilter(
      "Fir", R"({"commandQueue": "kat", "taps": [0.5, 1.0], "tapType": "Float",
                 "elementType": "FloatComplex", "decimation": 2})"));
  firTwoCommits(fir.get(), q.get());
  Result<Filter> fm = createFilter("QuadDemod", R"({"commandQueue": "kat", "modulation": "fm", "sampleRate": 1e6,
                                                    "fskDeviation": 5e3})");
  CHECK(fm.status == Status_Success && fm.value != nullptr);  // QuadFmDemod (QuadDemodFactory.h:91-110)
  if (fm.value != nullptr) fm.value->unref();
  Result<Filter> mul = createFilter("MultiplyCCC", R"({"commandQueue": "kat"})");
  CHECK(mul.status == Status_Success && mul.value != nullptr);
  if (mul.value != nullptr) mul.value->unref();
  ConstRef<Filter> am = unwrap(createFilter("QuadDemod", R"({"commandQueue": "kat", "modulation": "am"})"));
  CHECK(static_cast<Node*>(am.get())->asFilter() != nullptr);
  Result<Filter> bad = createFilter("Fir", "{not json");
  CHECK(bad.status == Status_ParseError);
  Result<Node> missing = createNode("NoSuchNode", "{}");
  CHECK(missing.status == Status_NotFound);
}

// Int8ToFloat -> Fir (127 taps, FC, D=3) -> QuadAmDemod through the Sink/Source contract, fed in
// uneven chunks and drained through deliberately small output buffers; compared with a double
// precision CPU evaluation of the same chain.
void chunkedChain(ICudaCommandQueue* q) {
  const size_t T = 127, D = 3;
  std::vector<float> taps(T);
  for (size_t j = 0; j < T; ++j) taps[j] = (float)(std::sin(0.37 * (double)j) / (double)T);
  ConstRef<Filter> conv = unwrap(F()->getInt8ToFloatFactory()->createFilter(q));
  ConstRef<Filter> fir =
      unwrap(F()->getFirFactory()->createFir(SampleType_Float, SampleType_FloatComplex, D, taps.data(), T, q));
  ConstRef<Filter> am = unwrap(F()->getQuadDemodFactory()->createQuadDemod(Modulation_Am, 1e6f, 0.0f, q));
  ConstRef<IAllocator> alloc = unwrap(F()->getCudaAllocatorFactory()->createCudaAllocator(q, 32, false));
  ConstRef<IBufferFactory> bf = unwrap(F()->createBufferFactory(alloc));

  const size_t nSamples = 50000;
  std::vector<int8_t> iq(2 * nSamples);
  uint32_t s = 12345;
  for (auto& v : iq) {
    s = s * 1664525u + 1013904223u;
    v = (int8_t)(s >> 24);
  }
  std::vector<float> amOut;
  const size_t chunks[] = {1, 4097, 333, 20000, 7, 25562};
  size_t pos = 0;
  auto pump = [&](Source* from, Sink* to, size_t cap) {
    // move everything available from `from` into `to` through a `cap`-byte device buffer
    for (;;) {
      const size_t avail = from->getOutputDataSize(0);
      if (avail == 0) return;
      ConstRef<IBuffer> tmp = unwrap(bf->createBuffer(cap));
      IBuffer* outs[] = {tmp.get()};
      THROW_IF_ERR(from->readOutput(outs, 1));
      if (tmp->range()->used() == 0) return;
      ConstRef<IBuffer> in = unwrap(to->requestBuffer(0, tmp->range()->used()));
      ConstRef<IBufferCopier> d2d = from->getOutputCopier(0);
      THROW_IF_ERR(d2d->copy(in->writePtr(), tmp->readPtr(), tmp->range()->used()));
      THROW_IF_ERR(to->commitBuffer(0, tmp->range()->used()));
    }
  };
  for (size_t c : chunks) {
    push(conv.get(), iq.data() + 2 * pos, 2 * c, q);
    pos += c;
    pump(conv.get(), fir.get(), 64 * 1024);
    pump(fir.get(), am.get(), 8 * 1000);  // not a multiple of the chunking: partial reads
    for (;;) {
      const size_t avail = am->getOutputDataSize(0);
      if (avail == 0) break;
      ConstRef<IBuffer> out = unwrap(bf->createBuffer(3000));
      IBuffer* outs[] = {out.get()};
      THROW_IF_ERR(am->readOutput(outs, 1));
      std::vector<uint8_t> h = toHost(out, q);
      const float* f = reinterpret_cast<const float*>(h.data());
      amOut.insert(amOut.end(), f, f + h.size() / sizeof(float));
    }
  }
  CHECK(pos == nSamples);
  const size_t expectN = (nSamples - (T - 1)) / D;  // Fir.cpp:178-186 over the whole stream
  CHECK(amOut.size() == expectN);
  size_t bad = 0;
  for (size_t k = 0; k < amOut.size() && k < expectN; ++k) {
    double re = 0, im = 0, bound = 0;
    for (size_t j = 0; j < T; ++j) {
      const size_t n = k * D + j;
      const double xr = std::max(-1.0, (double)(float)((float)iq[2 * n] / 127.0f));
      const double xi = std::max(-1.0, (double)(float)((float)iq[2 * n + 1] / 127.0f));
      re += taps[j] * xr;
      im += taps[j] * xi;
      bound += std::fabs(taps[j]) * std::hypot(xr, xi);
    }
    if (std::fabs(amOut[k] - std::hypot(re, im)) > 1e-6 * bound + 1e-30) ++bad;
  }
  CHECK(bad == 0);
}

void run(const char* name, const std::function<void()>& fn) {
  const int before = gFailures;
  try {
    fn();
  } catch (const std::exception& e) {
    fprintf(stderr, "%s threw: %s\n", name, e.what());
    ++gFailures;
  }
  printf("%-22s %s\n", name, gFailures == before ? "ok" : "FAILED");
}

}  // namespace

int main() {
  ConstRef<ICudaCommandQueue> q = unwrap(F()->getCudaCommandQueueFactory()->create(0));
  run("fir_two_commits", [&]() {
    const float taps[] = {0.5f, 1.0f};
    ConstRef<Filter> fir =
        unwrap(F()->getFirFactory()->createFir(SampleType_Float, SampleType_FloatComplex, 2, taps, 2, q));
    firTwoCommits(fir.get(), q.get());
  });
  run("fir_partial_reads", [&]() { firPartialReads(q.get()); });
  run("cosine_source", [&]() { cosineSource(q.get()); });
  run("json_registry", [&]() { jsonRegistry(); });
  run("chunked_chain", [&]() { chunkedChain(q.get()); });
  printf("%s (%d failures)\n", gFailures == 0 ? "ALL PASS" : "FAILURES", gFailures);
  return gFailures == 0 ? 0 : 1;
}
