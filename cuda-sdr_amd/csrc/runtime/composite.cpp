// Composite graphs: FilterDriver, the JSON "Component" factory, port remapping, RF -> PCM audio and
// the read-byte-count monitor. See composite.h for the reference files each one follows.
#include "composite.h"

#include <gpusdrpipeline/abi/errors.h>

#include <cmath>
#include <map>
#include <string>
#include <unordered_map>

#include "driver.h"
#include "json.h"

namespace gsdr_rt {

// ---- low-pass design ------------------------------------------------------------------------------------
namespace {
double besselI0(double x) {
  double sum = 1.0, term = 1.0;
  const double q = x * x / 4.0;
  for (int k = 1; k < 200; ++k) {
    term *= q / ((double)k * (double)k);
    sum += term;
    if (term < 1e-17 * sum) break;
  }
  return sum;
}
}  // namespace

Status designLowPass(double sampleRate, double cutoff, double transitionWidth, double dbAttenuation,
                     std::vector<float>& taps) noexcept {
  try {
    if (!(sampleRate > 0) || !(cutoff > 0) || !(transitionWidth > 0) || cutoff + transitionWidth > sampleRate / 2 ||
        dbAttenuation == 0.0) {
      gsloge("Low-pass design: need 0 < cutoff < cutoff + transition <= fs / 2 and a nonzero attenuation "
             "(fs %g, cutoff %g, transition %g, attenuation %g dB)",
             sampleRate, cutoff, transitionWidth, dbAttenuation);
      return Status_InvalidArgument;
    }
    const double att = std::fabs(dbAttenuation);  // the reference passes negative dB (RfToPcmAudioFactory.cpp:44-47)
    const double len = std::ceil(att / (22.0 * transitionWidth / sampleRate));
    if (!(len >= 3.0) || len > 1e6) {
      gsloge("Low-pass design: tap count %g out of range", len);
      return Status_InvalidArgument;
    }
    const size_t n = (size_t)len;
    const double beta = att > 50.0 ? 0.1102 * (att - 8.7)
                                   : (att >= 21.0 ? 0.5842 * std::pow(att - 21.0, 0.4) + 0.07886 * (att - 21.0) : 0.0);
    const double fc = (cutoff + transitionWidth / 2.0) / sampleRate;  // cycles per sample
    const double mid = (double)(n - 1) / 2.0;
    const double i0b = besselI0(beta);
    std::vector<double> h(n);
    double sum = 0.0;
    for (size_t i = 0; i < n; ++i) {
      const double t = (double)i - mid;
      const double ideal = t == 0.0 ? 2.0 * fc : std::sin(2.0 * M_PI * fc * t) / (M_PI * t);
      const double r = n > 1 ? 2.0 * t / (double)(n - 1) : 0.0;
      const double w = besselI0(beta * std::sqrt(std::max(0.0, 1.0 - r * r))) / i0b;
      h[i] = ideal * w;
      sum += h[i];
    }
    taps.resize(n);
    for (size_t i = 0; i < n; ++i) taps[i] = (float)(h[i] / sum);
    return Status_Success;
  }
  IF_CATCH_RETURN_STATUS;
}

namespace {

// ---- port remapping (PortRemappingSink.cpp, PortRemappingSource.cpp) -------------------------------------
class PortRemappingSink final : public IPortRemappingSink {
 public:
  void addPortMapping(size_t outerPort, Sink* innerSink, size_t innerSinkPort) noexcept final {
    try {
      mMap.erase(outerPort);
      mMap.emplace(outerPort, Mapped{innerSink, innerSinkPort});
    } catch (...) {
      gsloge("PortRemappingSink: out of memory adding port [%zu]", outerPort);
    }
  }
  Result<IBuffer> requestBuffer(size_t port, size_t byteCount) noexcept final {
    auto it = mMap.find(port);
    if (it == mMap.end()) {
      gsloge("Input port [%zu] is not mapped", port);
      return ERR_RESULT(Status_InvalidArgument);
    }
    return it->second.sink->requestBuffer(it->second.port, byteCount);
  }
  Status commitBuffer(size_t port, size_t byteCount) noexcept final {
    auto it = mMap.find(port);
    if (it == mMap.end()) {
      gsloge("Input port [%zu] is not mapped", port);
      return Status_InvalidArgument;
    }
    return it->second.sink->commitBuffer(it->second.port, byteCount);
  }
  // The reference aborts on an unmapped port (PortRemappingSink.cpp:48-50); 0 here, logged.
  size_t preferredInputBufferSize(size_t port) noexcept final {
    auto it = mMap.find(port);
    if (it == mMap.end()) {
      gsloge("Input port [%zu] is not mapped", port);
      return 0;
    }
    return it->second.sink->preferredInputBufferSize(it->second.port);
  }

 private:
  struct Mapped {
    ImmutableRef<Sink> sink;
    size_t port;
  };
  std::map<size_t, Mapped> mMap;
  REF_COUNTED(PortRemappingSink);
};

class PortRemappingSource final : public IPortRemappingSource {
 public:
  void addPortMapping(size_t outerPort, Source* innerSource, size_t innerSourcePort) noexcept final {
    try {
      mByOuter.erase(outerPort);
      mByOuter.emplace(outerPort, Mapped{innerSource, innerSourcePort});
      auto it = mBySource.find(innerSource);
      if (it == mBySource.end()) {
        mSourceOrder.emplace_back(innerSource);
        it = mBySource.emplace(innerSource, std::vector<std::pair<size_t, size_t>>()).first;
      }
      it->second.emplace_back(outerPort, innerSourcePort);
    } catch (...) {
      gsloge("PortRemappingSource: out of memory adding port [%zu]", outerPort);
    }
  }
  size_t getOutputDataSize(size_t port) noexcept final {
    auto it = mByOuter.find(port);
    if (it == mByOuter.end()) {
      gslogw("Cannot get output data size. Output port [%zu] is not mapped.", port);
      return 0;
    }
    return it->second.source->getOutputDataSize(it->second.port);
  }
  size_t getOutputSizeAlignment(size_t port) noexcept final {
    auto it = mByOuter.find(port);
    if (it == mByOuter.end()) {
      gslogw("Cannot get output size alignment. Output port [%zu] is not mapped.", port);
      return 1;
    }
    return it->second.source->getOutputSizeAlignment(it->second.port);
  }
  IBufferCopier* getOutputCopier(size_t port) noexcept final {
    auto it = mByOuter.find(port);
    return it == mByOuter.end() ? nullptr : it->second.source->getOutputCopier(it->second.port);
  }
  // PortRemappingSource.cpp:75-118: each inner source reads once, with the outer buffers of the
  // ports mapped to it placed at its inner port positions (every inner port up to the highest mapped
  // one must be mapped).
  Status readOutput(IBuffer** portOutputBuffers, size_t numPorts) noexcept final {
    try {
      for (Source* source : mSourceOrder) {
        const auto& maps = mBySource.at(source);
        std::vector<IBuffer*> inner;
        for (const auto& m : maps) {
          if (m.first >= numPorts) {
            gsloge("Too few output buffers: exposed port [%zu] is mapped, %zu buffers given", m.first, numPorts);
            return Status_InvalidArgument;
          }
          if (inner.size() <= m.second) inner.resize(m.second + 1, nullptr);
          inner[m.second] = portOutputBuffers[m.first];
        }
        for (size_t i = 0; i < inner.size(); ++i) {
          if (inner[i] == nullptr) {
            gsloge("Inner port [%zu] of a remapped source is not mapped to an exposed port", i);
            return Status_InvalidArgument;
          }
        }
        FWD_IF_ERR(source->readOutput(inner.data(), inner.size()));
      }
      return Status_Success;
    }
    IF_CATCH_RETURN_STATUS;
  }

 private:
  struct Mapped {
    ImmutableRef<Source> source;
    size_t port;
  };
  std::map<size_t, Mapped> mByOuter;
  std::vector<ImmutableRef<Source>> mSourceOrder;  // deterministic read order (an unordered_map in the reference)
  std::unordered_map<Source*, std::vector<std::pair<size_t, size_t>>> mBySource;  // (exposed, inner) ports
  REF_COUNTED(PortRemappingSource);
};

class PortRemappingSinkFactory final : public IPortRemappingSinkFactory {
 public:
  Result<IPortRemappingSink> create() noexcept final {
    return makeRefResultNonNull<IPortRemappingSink>(new (std::nothrow) PortRemappingSink());
  }
  REF_COUNTED(PortRemappingSinkFactory);
};

class PortRemappingSourceFactory final : public IPortRemappingSourceFactory {
 public:
  Result<IPortRemappingSource> create() noexcept final {
    return makeRefResultNonNull<IPortRemappingSource>(new (std::nothrow) PortRemappingSource());
  }
  REF_COUNTED(PortRemappingSourceFactory);
};

// ---- FilterDriver (FilterDriver.cpp) ------------------------------------------------------------------
// A Filter whose input is an inner node's sink (setDriverInput) and whose output is an inner node's
// source (setDriverOutput); committing input steps the inner graph once, and reading output steps it
// when the output node has nothing yet. MI355X extension: with a graph stream set (JSON
// "hipGraphCommandQueue"), each inner step runs through SteppingDriver::doFilterGraphed, so a
// component in steady state replays its whole step as one cached hipGraph.
class FilterDriver final : public IFilterDriver {
 public:
  explicit FilterDriver(ISteppingDriver* stepping) noexcept : mStepping(stepping) {}

  void setGraphStream(hipStream_t stream) noexcept { mGraphStream = stream; }
  SteppingDriver* stepping() const noexcept { return dynamic_cast<SteppingDriver*>(mStepping.get()); }

  void setDriverInput(Sink* sink) noexcept final { mInput = sink; }
  void setDriverOutput(Source* source) noexcept final { mOutput = source; }

  Status connect(Source* source, size_t sourcePort, Sink* sink, size_t sinkPort) noexcept final {
    return mStepping->connect(source, sourcePort, sink, sinkPort);
  }
  Status setupNode(Node* node, const char* functionInGraph) noexcept final {
    return mStepping->setupNode(node, functionInGraph);
  }

  void iterateOverConnections(void* context,
                              void (*it)(IDriver* driver, void* context, Source* source, size_t sourcePort, Sink* sink,
                                         size_t sinkPort) noexcept) noexcept final {
    Callback cb{this, context, it, nullptr, nullptr};
    mStepping->iterateOverConnections(&cb, [](IDriver*, void* c, Source* so, size_t sp, Sink* si, size_t kp) noexcept {
      auto* cb = static_cast<Callback*>(c);
      cb->conn(cb->self, cb->context, so, sp, si, kp);
    });
    // FilterDriver.cpp:120-126: the delegates as edges of this node
    Ref<Sink> in(mInput);
    Ref<Source> out(mOutput);
    if (in != nullptr) it(this, context, this, 0, in.get(), 0);
    if (out != nullptr) it(this, context, out.get(), 0, this, 0);
  }
  void iterateOverNodes(void* context, void (*it)(IDriver* driver, void* context, Node* node) noexcept) noexcept final {
    Callback cb{this, context, nullptr, it, nullptr};
    mStepping->iterateOverNodes(&cb, [](IDriver*, void* c, Node* n) noexcept {
      auto* cb = static_cast<Callback*>(c);
      cb->node(cb->self, cb->context, n);
    });
  }
  void iterateOverNodeAttributes(Node* node, void* context,
                                 void (*it)(IDriver* driver, Node* node, void* context, const char* attrName,
                                            const char* attrVal) noexcept) noexcept final {
    Callback cb{this, context, nullptr, nullptr, it};
    mStepping->iterateOverNodeAttributes(node, &cb, [](IDriver*, Node* n, void* c, const char* k, const char* v) noexcept {
      auto* cb = static_cast<Callback*>(c);
      cb->attr(cb->self, n, cb->context, k, v);
    });
    if (node == nullptr) return;
    Ref<Sink> in(mInput);
    Ref<Source> out(mOutput);
    if (in != nullptr && node->asSink() == in.get().get()) it(this, node, context, "inputNode", "true");
    if (out != nullptr && node->asSource() == out.get().get()) it(this, node, context, "outputNode", "true");
  }
  size_t getNodeName(Node* node, char* name, size_t nameBufLen, bool* foundOut) noexcept final {
    return mStepping->getNodeName(node, name, nameBufLen, foundOut);
  }

  // ---- Sink side --------------------------------------------------------------------------------------
  Result<IBuffer> requestBuffer(size_t port, size_t byteCount) noexcept final {
    Ref<Sink> in(mInput);
    if (in == nullptr) {
      gsloge("Cannot use FilterDriver as a Sink until a node is set via setDriverInput()");
      return ERR_RESULT(Status_InvalidState);
    }
    return in->requestBuffer(port, byteCount);
  }
  Status commitBuffer(size_t port, size_t byteCount) noexcept final {
    Ref<Sink> in(mInput);
    if (in == nullptr) {
      gsloge("Cannot use FilterDriver as a Sink until a node is set via setDriverInput()");
      return Status_InvalidState;
    }
    FWD_IF_ERR(in->commitBuffer(port, byteCount));
    return step();
  }
  // The reference dereferences a null delegate here (FilterDriver.cpp:290-294); 0 / null, logged.
  size_t preferredInputBufferSize(size_t port) noexcept final {
    Ref<Sink> in(mInput);
    if (in == nullptr) {
      gsloge("FilterDriver has no input node (setDriverInput)");
      return 0;
    }
    return in->preferredInputBufferSize(port);
  }

  // ---- Source side ------------------------------------------------------------------------------------
  size_t getOutputDataSize(size_t port) noexcept final {
    Ref<Source> out(mOutput);
    if (out == nullptr) {
      gslogw("Cannot use FilterDriver as a Source until a node is set via setDriverOutput()");
      return 0;
    }
    if (out->getOutputDataSize(port) == 0 && step() != Status_Success) return 0;
    return out->getOutputDataSize(port);
  }
  size_t getOutputSizeAlignment(size_t port) noexcept final {
    Ref<Source> out(mOutput);
    if (out == nullptr) {
      gslogw("Cannot use FilterDriver as a Source until a node is set via setDriverOutput()");
      return 1;
    }
    return out->getOutputSizeAlignment(port);
  }
  IBufferCopier* getOutputCopier(size_t port) noexcept final {
    Ref<Source> out(mOutput);
    return out == nullptr ? nullptr : out->getOutputCopier(port);
  }
  Status readOutput(IBuffer** portOutputBuffers, size_t numPorts) noexcept final {
    Ref<Source> out(mOutput);
    if (out == nullptr) {
      gsloge("Cannot use FilterDriver as a Source until a node is set via setDriverOutput()");
      return Status_InvalidState;
    }
    bool all = true;
    for (size_t p = 0; p < numPorts; ++p) all = all && out->getOutputDataSize(p) != 0;
    if (!all) FWD_IF_ERR(step());
    return out->readOutput(portOutputBuffers, numPorts);
  }

 private:
  Status step() noexcept {
    if (mGraphStream != nullptr) {
      if (SteppingDriver* d = stepping()) return d->doFilterGraphed(mGraphStream);
    }
    return mStepping->doFilter();
  }
  struct Callback {
    FilterDriver* self;
    void* context;
    void (*conn)(IDriver*, void*, Source*, size_t, Sink*, size_t) noexcept;
    void (*node)(IDriver*, void*, Node*) noexcept;
    void (*attr)(IDriver*, Node*, void*, const char*, const char*) noexcept;
  };
  ConstRef<ISteppingDriver> mStepping;
  Ref<Sink> mInput;
  Ref<Source> mOutput;
  hipStream_t mGraphStream = nullptr;
  REF_COUNTED(FilterDriver);
};

// ---- the JSON "Component" factory (FilterDriverFactory.cpp:27-178) -------------------------------------
// {
//   "nodes": {"<id>": {"type": "<registered node type>", ...node parameters...}, ...},
//   "connections": [{"source": id, "sourcePort": n, "sink": id, "sinkPort": n}, ...],
//   "inputPorts": [{"exposedPort": n, "mapped": {"node": id, "port": n}}, ...],
//   "outputPorts": [{"exposedPort": n, "mapped": {"node": id, "port": n}}, ...]
// }
// Differences from the reference, all deliberate: each node is created from ITS OWN definition
// (the reference passes the whole component text to every node, FilterDriverFactory.cpp:51);
// "sourcePort" / "sinkPort" default to 0 and "target" / "targetPort" are accepted for "sink" /
// "sinkPort" (the forms RfToPcmAudioFactory.cpp:270-292 and the header comment use); "outputPort":
// "<id>" maps exposed port 0 to that node's port 0 (RfToPcmAudioFactory.cpp:304); every node is
// named in the driver with its id (setupNode), so drivers can report it.
class FilterDriverFactory final : public IFilterDriverFactory {
 public:
  explicit FilterDriverFactory(IFactories* f) noexcept : mF(f) {}

  Result<IFilterDriver> createFilterDriver() noexcept final {
    Ref<ISteppingDriver> stepping;
    UNWRAP_OR_FWD_RESULT(stepping, mF->getSteppingDriverFactory()->createSteppingDriver());
    return makeRefResultNonNull<IFilterDriver>(new (std::nothrow) FilterDriver(stepping.get().get()));
  }

  Result<Node> create(const char* jsonParameters) noexcept final {
    try {
      Json params;
      std::string err;
      if (!Json::parse(jsonParameters, params, err) || !params.isObject()) {
        gsloge("Cannot parse component definition: %s", err.c_str());
        return ERR_RESULT(Status_ParseError);
      }
      const Json* nodeDefs = params.get("nodes");
      if (nodeDefs == nullptr || !nodeDefs->isObject()) {
        gsloge("Component definition needs a \"nodes\" object");
        return ERR_RESULT(Status_ParseError);
      }
      // the nodes come from the registry: register the defaults if nobody has
      if (!hasNodeFactory("Fir")) FWD_IN_RESULT_IF_ERR(registerDefaultNodeFactories());
      // The component stays floating until it is handed back (a Ref here would delete it when the
      // Ref dies on return); any failure below releases it.
      RefResult<IFilterDriver> created = createFilterDriver();
      if (created.status != Status_Success) return ERR_RESULT(created.status);
      struct Release {
        IFilterDriver* p;
        ~Release() {
          if (p != nullptr) p->unref();
        }
      } guard{created.value};
      IFilterDriver* const component = created.value;

      std::map<std::string, ImmutableRef<Node>> nodes;
      for (const auto& kv : nodeDefs->object()) {
        const Json* type = kv.second.get("type");
        if (type == nullptr || !type->isString()) {
          gsloge("Node definition for [%s] does not contain a type.", kv.first.c_str());
          return ERR_RESULT(Status_InvalidArgument);
        }
        Ref<Node> node;
        UNWRAP_OR_FWD_RESULT(node, createNode(type->string().c_str(), kv.second.dump().c_str()));
        nodes.emplace(kv.first, node.get().get());
        FWD_IN_RESULT_IF_ERR(component->setupNode(node.get().get(), kv.first.c_str()));
      }
      auto find = [&](const std::string& id) -> Node* {
        auto it = nodes.find(id);
        return it == nodes.end() ? nullptr : it->second.get();
      };
      auto str = [](const Json& j, const char* a, const char* b) -> const Json* {
        const Json* v = j.get(a);
        return v != nullptr ? v : (b != nullptr ? j.get(b) : nullptr);
      };
      auto num = [](const Json* j, size_t dflt) -> size_t {
        return j != nullptr && j->isNumber() && j->number() >= 0 ? (size_t)j->number() : dflt;
      };
      auto mapping = [&](const Json& m, std::string& nodeId, size_t& exposed, size_t& inner) {
        const Json* mapped = m.get("mapped");
        const Json* id = mapped != nullptr ? mapped->get("node") : nullptr;
        if (id == nullptr || !id->isString()) return false;
        nodeId = id->string();
        exposed = num(m.get("exposedPort"), 0);
        inner = num(mapped->get("port"), 0);
        return true;
      };

      if (const Json* ins = params.get("inputPorts"); ins != nullptr && ins->isArray() && !ins->array().empty()) {
        Ref<IPortRemappingSink> mapper;
        UNWRAP_OR_FWD_RESULT(mapper, mF->getPortRemappingSinkFactory()->create());
        for (const Json& m : ins->array()) {
          std::string id;
          size_t exposed, inner;
          if (!mapping(m, id, exposed, inner)) return ERR_RESULT(Status_ParseError);
          Node* n = find(id);
          if (n == nullptr) {
            gsloge("Cannot add an input port mapping with node [%s] because it was not defined.", id.c_str());
            return ERR_RESULT(Status_NotFound);
          }
          if (n->asSink() == nullptr) {
            gsloge("Cannot add an input port mapping with node [%s] because it is not a sink.", id.c_str());
            return ERR_RESULT(Status_InvalidArgument);
          }
          mapper->addPortMapping(exposed, n->asSink(), inner);
        }
        component->setDriverInput(mapper.get().get());
      }

      Ref<IPortRemappingSource> outMapper;
      auto mapOutput = [&](const std::string& id, size_t exposed, size_t inner) -> Status {
        Node* n = find(id);
        if (n == nullptr) {
          gsloge("Cannot add an output port mapping with node [%s] because it was not defined.", id.c_str());
          return Status_NotFound;
        }
        if (n->asSource() == nullptr) {
          gsloge("Cannot add an output port mapping with node [%s] because it is not a source.", id.c_str());
          return Status_InvalidArgument;
        }
        if (outMapper == nullptr) {
          Ref<IPortRemappingSource> m;
          UNWRAP_OR_FWD_STATUS(m, mF->getPortRemappingSourceFactory()->create());
          outMapper = m;
        }
        outMapper->addPortMapping(exposed, n->asSource(), inner);
        return Status_Success;
      };
      if (const Json* outs = params.get("outputPorts"); outs != nullptr && outs->isArray()) {
        for (const Json& m : outs->array()) {
          std::string id;
          size_t exposed, inner;
          if (!mapping(m, id, exposed, inner)) return ERR_RESULT(Status_ParseError);
          FWD_IN_RESULT_IF_ERR(mapOutput(id, exposed, inner));
        }
      }
      if (const Json* out = params.get("outputPort"); out != nullptr && out->isString()) {
        FWD_IN_RESULT_IF_ERR(mapOutput(out->string(), 0, 0));
      }
      if (outMapper != nullptr) component->setDriverOutput(outMapper.get().get());
      // MI355X extension: replay the inner graph's steady-state steps as hipGraphs on this queue
      if (const Json* gq = params.get("hipGraphCommandQueue"); gq != nullptr) {
        if (!gq->isString()) {
          gsloge("\"hipGraphCommandQueue\" must name a command queue");
          return ERR_RESULT(Status_ParseError);
        }
        Ref<ICudaCommandQueue> queue;
        UNWRAP_OR_FWD_RESULT(queue, mF->getCommandQueueFactory()->getCudaCommandQueue(gq->string().c_str()));
        static_cast<FilterDriver*>(component)->setGraphStream(queue->cudaStream());
      }

      if (const Json* conns = params.get("connections"); conns != nullptr && conns->isArray()) {
        for (const Json& c : conns->array()) {
          const Json* so = str(c, "source", nullptr);
          const Json* si = str(c, "sink", "target");
          if (so == nullptr || si == nullptr || !so->isString() || !si->isString()) {
            gsloge("A connection needs \"source\" and \"sink\" node ids");
            return ERR_RESULT(Status_ParseError);
          }
          const size_t sp = num(c.get("sourcePort"), 0);
          const size_t kp = num(str(c, "sinkPort", "targetPort"), 0);
          Node* src = find(so->string());
          Node* snk = find(si->string());
          if (src == nullptr || snk == nullptr) {
            gsloge("Cannot connect source [%s] port [%zu] to sink [%s] port [%zu]. %s is not defined.",
                   so->string().c_str(), sp, si->string().c_str(), kp, src == nullptr ? "Source" : "Sink");
            return ERR_RESULT(Status_InvalidArgument);
          }
          if (src->asSource() == nullptr || snk->asSink() == nullptr) {
            gsloge("Cannot connect source [%s] port [%zu] to sink [%s] port [%zu]. [%s] is not a %s.",
                   so->string().c_str(), sp, si->string().c_str(), kp,
                   src->asSource() == nullptr ? so->string().c_str() : si->string().c_str(),
                   src->asSource() == nullptr ? "source" : "sink");
            return ERR_RESULT(Status_InvalidArgument);
          }
          FWD_IN_RESULT_IF_ERR(component->connect(src->asSource(), sp, snk->asSink(), kp));
        }
      }
      guard.p = nullptr;
      return makeRefResultNonNull<Node>(component);
    }
    IF_CATCH_RETURN_RESULT;
  }

 private:
  IFactories* const mF;
  REF_COUNTED(FilterDriverFactory);
};

// ---- RF -> PCM audio (RfToPcmAudioFactory.cpp:129-317) ---------------------------------------------
// Differences from the reference, all deliberate: the node types are the registered ones ("Cosine",
// "MultiplyCCC"; the reference emits "Multiply", which no factory is registered under), "modulation"
// is the string the QuadDemod factory parses ("am" / "fm"; the reference emits the enum's number),
// the connections name the mixer's tone port, the taps come from designLowPass (composite.h), and
// the audio low-pass is designed at the rate it runs at (the demodulator's; the reference designs
// it at the audio output rate, RfToPcmAudioFactory.cpp:180-185, which puts its band edges 1 / D too
// high for the filter that actually runs).
class RfToPcmAudioFactory final : public IRfToPcmAudioFactory {
 public:
  explicit RfToPcmAudioFactory(IFactories* f) noexcept : mF(f) {}

  Result<Node> create(const char* jsonParameters) noexcept final {
    try {
      Json p;
      std::string err;
      if (!Json::parse(jsonParameters, p, err) || !p.isObject()) {
        gsloge("Cannot parse RF -> PCM parameters: %s", err.c_str());
        return ERR_RESULT(Status_ParseError);
      }
      auto num = [&](const char* k, double& out) {
        const Json* j = p.get(k);
        if (j == nullptr || !j->isNumber()) {
          gsloge("RF -> PCM parameters need a number \"%s\"", k);
          return false;
        }
        out = j->number();
        return true;
      };
      const Json* m = p.get("modulation");
      const Json* q = p.get("commandQueue");
      if (q == nullptr) q = p.get("commandQueueId");
      if (m == nullptr || !m->isString() || q == nullptr || !q->isString()) {
        gsloge("RF -> PCM parameters need \"modulation\" and \"commandQueue\" strings");
        return ERR_RESULT(Status_ParseError);
      }
      Modulation mod;
      if (m->string() == "am") mod = Modulation_Am;
      else if (m->string() == "fm") mod = Modulation_Fm;
      else {
        gsloge("Modulation [%s] is not supported. Supported modulations: 'fm', 'am'", m->string().c_str());
        return ERR_RESULT(Status_NotFound);
      }
      double rfRate, rfDecim, audioDecim, tuned, channel, width, rfAtt, audioAtt, dev = 0.0;
      if (!num("rfSampleRate", rfRate) || !num("rfLowPassDecimation", rfDecim) ||
          !num("audioLowPassDecimation", audioDecim) || !num("tunedFrequency", tuned) ||
          !num("channelFrequency", channel) || !num("channelWidth", width) ||
          !num("rfLowPassDbAttenuation", rfAtt) || !num("audioLowPassDbAttenuation", audioAtt))
        return ERR_RESULT(Status_ParseError);
      if (mod == Modulation_Fm && !num("fskDeviation", dev)) return ERR_RESULT(Status_ParseError);
      return ResultCast<Node>(createRfToPcm((float)rfRate, mod, (size_t)rfDecim, (size_t)audioDecim, (float)tuned,
                                            (float)channel, (float)width, (float)dev, (float)rfAtt, (float)audioAtt,
                                            q->string().c_str()));
    }
    IF_CATCH_RETURN_RESULT;
  }

  Result<Filter> createRfToPcm(float rfSampleRate, Modulation modulation, size_t rfLowPassDecim,
                               size_t audioLowPassDecim, float tunedFrequency, float channelFrequency,
                               float channelWidth, float fskDeviationIfFm, float rfLowPassDbAttenuation,
                               float audioLowPassDbAttenuation, const char* commandQueueId) noexcept final {
    try {
      if (rfLowPassDecim == 0 || audioLowPassDecim == 0 || commandQueueId == nullptr) {
        gsloge("RF -> PCM needs nonzero decimations and a command queue id");
        return ERR_RESULT(Status_InvalidArgument);
      }
      // RfToPcmAudioFactory.cpp:164-171 (same float expressions)
      const float audioRate =
          rfSampleRate / static_cast<float>(rfLowPassDecim) / static_cast<float>(audioLowPassDecim);
      const float demodRate = rfSampleRate / static_cast<float>(rfLowPassDecim);
      const float rfCutoff = demodRate / 2.0f * 0.95f;
      const float rfTransition = demodRate / 2.0f * 0.05f;
      const float audioCutoff = audioRate / 2.0f * 0.9f;
      const float audioTransition = audioRate / 2.0f * 0.1f;
      std::vector<float> rfTaps, audioTaps;
      FWD_IN_RESULT_IF_ERR(designLowPass(rfSampleRate, rfCutoff, rfTransition, rfLowPassDbAttenuation, rfTaps));
      // the audio FIR runs at the demodulator's rate; its band edges are the audio rate's
      FWD_IN_RESULT_IF_ERR(designLowPass(demodRate, audioCutoff, audioTransition, audioLowPassDbAttenuation, audioTaps));
      gslogd("RF -> PCM: RF low-pass %zu taps D %zu, audio low-pass %zu taps D %zu, tone %f Hz", rfTaps.size(),
             rfLowPassDecim, audioTaps.size(), audioLowPassDecim, tunedFrequency - channelFrequency);

      auto arr = [](const std::vector<float>& v) {
        std::string s = "[";
        char buf[32];
        for (size_t i = 0; i < v.size(); ++i) {
          snprintf(buf, sizeof(buf), "%s%.9g", i ? "," : "", (double)v[i]);
          s += buf;
        }
        return s + "]";
      };
      std::string qs = "\"";  // the queue id as a JSON string literal
      for (const char* c = commandQueueId; *c; ++c) {
        if (*c == '"' || *c == '\\') qs += '\\';
        qs += *c;
      }
      qs += '"';
      char head[1024];
      snprintf(head, sizeof(head),
               "{\"nodes\":{"
               "\"cosineSource\":{\"type\":\"Cosine\",\"sampleType\":\"FloatComplex\",\"sampleRate\":%.17g,"
               "\"frequency\":%.17g,\"commandQueue\":%s},"
               "\"multiplyForFrequencyShift\":{\"type\":\"MultiplyCCC\",\"commandQueue\":%s},"
               "\"quadDemod\":{\"type\":\"QuadDemod\",\"modulation\":\"%s\",\"sampleRate\":%.17g,"
               "\"fskDeviation\":%.17g,\"commandQueue\":%s},",
               (double)rfSampleRate, (double)(tunedFrequency - channelFrequency), qs.c_str(), qs.c_str(),
               modulation == Modulation_Fm ? "fm" : "am", (double)demodRate, (double)fskDeviationIfFm, qs.c_str());
      std::string def = head;
      def += "\"rfLowPassFilter\":{\"type\":\"Fir\",\"tapType\":\"Float\",\"elementType\":\"FloatComplex\","
             "\"decimation\":" + std::to_string(rfLowPassDecim) + ",\"commandQueue\":" + qs +
             ",\"taps\":" + arr(rfTaps) + "},";
      def += "\"audioLowPassFilter\":{\"type\":\"Fir\",\"tapType\":\"Float\",\"elementType\":\"Float\","
             "\"decimation\":" + std::to_string(audioLowPassDecim) + ",\"commandQueue\":" + qs +
             ",\"taps\":" + arr(audioTaps) + "}},";
      def += "\"connections\":["
             "{\"source\":\"cosineSource\",\"sink\":\"multiplyForFrequencyShift\",\"sinkPort\":1},"
             "{\"source\":\"multiplyForFrequencyShift\",\"sink\":\"rfLowPassFilter\"},"
             "{\"source\":\"rfLowPassFilter\",\"sink\":\"quadDemod\"},"
             "{\"source\":\"quadDemod\",\"sink\":\"audioLowPassFilter\"}],"
             "\"inputPorts\":[{\"exposedPort\":0,\"mapped\":{\"node\":\"multiplyForFrequencyShift\",\"port\":0}}],"
             "\"outputPort\":\"audioLowPassFilter\"}";
      // handed on floating (a Ref here would free it on return)
      RefResult<Node> created = mF->getFilterDriverFactory()->create(def.c_str());
      if (created.status != Status_Success) return ERR_RESULT(created.status);
      Filter* f = created.value->asFilter();
      if (f == nullptr) {
        created.value->unref();
        gsloge("RF -> PCM Audio component is not a filter");
        return ERR_RESULT(Status_RuntimeError);
      }
      return makeRefResultNonNull<Filter>(f);
    }
    IF_CATCH_RETURN_RESULT;
  }

 private:
  IFactories* const mF;
  REF_COUNTED(RfToPcmAudioFactory);
};

// ---- ReadByteCountMonitor (ReadByteCountMonitor.cpp) ----------------------------------------------------
// Forwards every call to the monitored filter and counts the bytes each readOutput added to each
// output buffer.
class ReadByteCountMonitor final : public IReadByteCountMonitor {
 public:
  explicit ReadByteCountMonitor(Filter* filter) noexcept : mFilter(filter) {}
  size_t getByteCountRead(size_t port) noexcept final { return port < mTotal.size() ? mTotal[port] : 0; }
  Result<IBuffer> requestBuffer(size_t port, size_t byteCount) noexcept final {
    return mFilter->requestBuffer(port, byteCount);
  }
  Status commitBuffer(size_t port, size_t byteCount) noexcept final { return mFilter->commitBuffer(port, byteCount); }
  size_t preferredInputBufferSize(size_t port) noexcept final { return mFilter->preferredInputBufferSize(port); }
  size_t getOutputDataSize(size_t port) noexcept final { return mFilter->getOutputDataSize(port); }
  size_t getOutputSizeAlignment(size_t port) noexcept final { return mFilter->getOutputSizeAlignment(port); }
  IBufferCopier* getOutputCopier(size_t port) noexcept final { return mFilter->getOutputCopier(port); }
  Status readOutput(IBuffer** portOutputBuffers, size_t numPorts) noexcept final {
    try {
      if (mTotal.size() < numPorts) {
        mTotal.resize(numPorts, 0);
        mBefore.resize(numPorts, 0);
      }
      for (size_t p = 0; p < numPorts; ++p) mBefore[p] = portOutputBuffers[p]->range()->used();
      FWD_IF_ERR(mFilter->readOutput(portOutputBuffers, numPorts));
      for (size_t p = 0; p < numPorts; ++p) mTotal[p] += portOutputBuffers[p]->range()->used() - mBefore[p];
      return Status_Success;
    }
    IF_CATCH_RETURN_STATUS;
  }

 private:
  ConstRef<Filter> mFilter;
  std::vector<size_t> mTotal;
  std::vector<size_t> mBefore;
  REF_COUNTED(ReadByteCountMonitor);
};

class ReadByteCountMonitorFactory final : public IReadByteCountMonitorFactory {
 public:
  Result<IReadByteCountMonitor> create(Filter* monitoredFilter) noexcept final {
    if (monitoredFilter == nullptr) return ERR_RESULT(Status_InvalidArgument);
    return makeRefResultNonNull<IReadByteCountMonitor>(new (std::nothrow) ReadByteCountMonitor(monitoredFilter));
  }
  REF_COUNTED(ReadByteCountMonitorFactory);
};

}  // namespace

IFilterDriverFactory* newFilterDriverFactory(IFactories* f) noexcept { return new (std::nothrow) FilterDriverFactory(f); }
SteppingDriver* componentSteppingDriver(IDriver* driver) noexcept {
  auto* fd = dynamic_cast<FilterDriver*>(driver);
  return fd == nullptr ? nullptr : fd->stepping();
}
IPortRemappingSinkFactory* newPortRemappingSinkFactory() noexcept { return new (std::nothrow) PortRemappingSinkFactory(); }
IPortRemappingSourceFactory* newPortRemappingSourceFactory() noexcept {
  return new (std::nothrow) PortRemappingSourceFactory();
}
IRfToPcmAudioFactory* newRfToPcmAudioFactory(IFactories* f) noexcept { return new (std::nothrow) RfToPcmAudioFactory(f); }
IReadByteCountMonitorFactory* newReadByteCountMonitorFactory() noexcept {
  return new (std::nothrow) ReadByteCountMonitorFactory();
}

}  // namespace gsdr_rt
