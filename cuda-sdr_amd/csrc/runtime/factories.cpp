// IFactories singleton, node factories and the node registry (reference src/Factories.cpp:63-204,
// src/filters/FilterFactories.cpp:23-150, src/filters/factories/*.h).
#include <gpusdrpipeline/Factories.h>

#include <mutex>
#include <string>
#include <unordered_map>

#include "buffers.h"
#include "composite.h"
#include "driver.h"
#include "filters.h"
#include "json.h"
#include "queues.h"

namespace gsdr_rt {

namespace {

// ParseJson.h:160-180
bool parseSampleType(const Json* j, SampleType& out) {
  if (j == nullptr || !j->isString()) return false;
  const std::string& s = j->string();
  if (s == "FloatComplex") out = SampleType_FloatComplex;
  else if (s == "Float") out = SampleType_Float;
  else if (s == "Int8Complex") out = SampleType_Int8Complex;
  else return false;
  return true;
}

bool parseParams(const char* json, Json& out) {
  std::string err;
  if (!Json::parse(json, out, err) || !out.isObject()) {
    gsloge("Cannot parse node parameters [%s]: %s", json ? json : "(null)", err.c_str());
    return false;
  }
  return true;
}

// "commandQueue" (FirFactory.h:32) or "commandQueueId" (the key RfToPcmAudioFactory.cpp:241-245 emits)
Result<ICudaCommandQueue> queueFromParams(IFactories* f, const Json& params) {
  const Json* q = params.get("commandQueue");
  if (q == nullptr) q = params.get("commandQueueId");
  if (q == nullptr || !q->isString()) {
    gsloge("Node parameters need a \"commandQueue\" string");
    return ERR_RESULT(Status_InvalidArgument);
  }
  return f->getCommandQueueFactory()->getCudaCommandQueue(q->string().c_str());
}

const char* kOutOfScope = "is outside this build's scope (FIR -> QuadAmDemod hot path; DESIGN.md)";

}  // namespace

// ---- in-scope node factories ------------------------------------------------------------------------------
class FirFactory final : public IFirFactory {
 public:
  explicit FirFactory(IFactories* f) noexcept : mF(f) {}
  Result<Node> create(const char* jsonParameters) noexcept final {
    try {
      Json p;
      if (!parseParams(jsonParameters, p)) return ERR_RESULT(Status_ParseError);
      Ref<ICudaCommandQueue> q;
      UNWRAP_OR_FWD_RESULT(q, queueFromParams(mF, p));
      SampleType tapType, elemType;
      const Json* et = p.get("elementType");
      if (et == nullptr) et = p.get("signalType");
      if (!parseSampleType(p.get("tapType"), tapType) || !parseSampleType(et, elemType)) {
        gsloge("Fir needs \"tapType\" and \"elementType\" in {Float, FloatComplex, Int8Complex}");
        return ERR_RESULT(Status_ParseError);
      }
      const Json* taps = p.get("taps");
      if (taps == nullptr || !taps->isArray()) return ERR_RESULT(Status_ParseError);
      std::vector<float> t;
      for (const Json& v : taps->array()) {
        if (v.isNumber()) {
          t.push_back((float)v.number());
        } else if (v.isArray() && v.array().size() == 2) {  // complex tap as [re, im]
          t.push_back((float)v.array()[0].number());
          t.push_back((float)v.array()[1].number());
        } else {
          return ERR_RESULT(Status_ParseError);
        }
      }
      size_t count = t.size();
      if (tapType == SampleType_FloatComplex) count /= 2;
      const Json* d = p.get("decimation");
      const size_t decim = d != nullptr && d->isNumber() ? (size_t)d->number() : 1;
      return ResultCast<Node>(createFir(tapType, elemType, decim, t.data(), count, q.get().get()));
    }
    IF_CATCH_RETURN_RESULT;
  }
  Result<Filter> createFir(SampleType tapType, SampleType elementType, size_t decimation, const float* taps,
                           size_t tapCount, ICudaCommandQueue* queue) noexcept final {
    return Fir::create(tapType, elementType, decimation, taps, tapCount, queue, mF);
  }

 private:
  IFactories* const mF;  // the immortal singleton
  REF_COUNTED(FirFactory);
};

class QuadDemodFactory final : public IQuadDemodFactory {
 public:
  explicit QuadDemodFactory(IFactories* f) noexcept : mF(f) {}
  Result<Node> create(const char* jsonParameters) noexcept final {
    try {
      Json p;
      if (!parseParams(jsonParameters, p)) return ERR_RESULT(Status_ParseError);
      const Json* m = p.get("modulation");
      if (m == nullptr || !m->isString()) return ERR_RESULT(Status_ParseError);
      Modulation mod;
      if (m->string() == "am") mod = Modulation_Am;
      else if (m->string() == "fm") mod = Modulation_Fm;
      else {
        gsloge("Modulation [%s] is not supported. Supported modulations: 'fm', 'am'", m->string().c_str());
        return ERR_RESULT(Status_NotFound);
      }
      const Json* sr = p.get("sampleRate");
      const Json* dev = p.get("fskDeviation");
      Ref<ICudaCommandQueue> q;
      UNWRAP_OR_FWD_RESULT(q, queueFromParams(mF, p));
      return ResultCast<Node>(createQuadDemod(mod, sr && sr->isNumber() ? (float)sr->number() : 0.0f,
                                              dev && dev->isNumber() ? (float)dev->number() : 0.0f, q.get().get()));
    }
    IF_CATCH_RETURN_RESULT;
  }
  // QuadDemodFactory.h:111 (same float expression)
  static float quadDemodGain(float inputSampleRate, float fskDeviation) noexcept {
    return inputSampleRate / (2.0f * 3.14159265358979323846f * fskDeviation * 5);
  }
  Result<Filter> createQuadDemod(Modulation modulation, float rfSampleRate, float fskDeviation,
                                 ICudaCommandQueue* queue) noexcept final {
    if (modulation == Modulation_Am) return QuadAmDemod::create(queue, mF);
    if (modulation == Modulation_Fm) {
      if (!(fskDeviation > 0.0f)) {
        gsloge("FM demodulation needs fskDeviation > 0 (got %f)", fskDeviation);
        return ERR_RESULT(Status_InvalidArgument);
      }
      return QuadFmDemod::create(quadDemodGain(rfSampleRate, fskDeviation), queue, mF);
    }
    gsloge("Modulation [%u] is not supported", modulation);
    return ERR_RESULT(Status_InvalidArgument);
  }

 private:
  IFactories* const mF;
  REF_COUNTED(QuadDemodFactory);
};

// Int8ToFloat (Int8ToFloatFactory.h) and Magnitude (|z|: the AM envelope kernel).
class QueueFilterFactory final : public ICudaFilterFactory {
 public:
  using Creator = Result<Filter> (*)(ICudaCommandQueue*, IFactories*) noexcept;
  QueueFilterFactory(IFactories* f, Creator c) noexcept : mF(f), mCreate(c) {}
  Result<Node> create(const char* jsonParameters) noexcept final {
    try {
      Json p;
      if (!parseParams(jsonParameters, p)) return ERR_RESULT(Status_ParseError);
      Ref<ICudaCommandQueue> q;
      UNWRAP_OR_FWD_RESULT(q, queueFromParams(mF, p));
      return ResultCast<Node>(createFilter(q.get().get()));
    }
    IF_CATCH_RETURN_RESULT;
  }
  Result<Filter> createFilter(ICudaCommandQueue* queue) noexcept final { return mCreate(queue, mF); }

 private:
  IFactories* const mF;
  const Creator mCreate;
  REF_COUNTED(QueueFilterFactory);
};

class CosineSourceFactory final : public ICosineSourceFactory {
 public:
  explicit CosineSourceFactory(IFactories* f) noexcept : mF(f) {}
  Result<Node> create(const char* jsonParameters) noexcept final {
    try {
      Json p;
      if (!parseParams(jsonParameters, p)) return ERR_RESULT(Status_ParseError);
      Ref<ICudaCommandQueue> q;
      UNWRAP_OR_FWD_RESULT(q, queueFromParams(mF, p));
      SampleType t;
      if (!parseSampleType(p.get("sampleType"), t)) return ERR_RESULT(Status_ParseError);
      const Json* sr = p.get("sampleRate");
      const Json* fr = p.get("frequency");
      if (sr == nullptr || fr == nullptr) return ERR_RESULT(Status_ParseError);
      return ResultCast<Node>(createCosineSource(t, (float)sr->number(), (float)fr->number(), q.get().get()));
    }
    IF_CATCH_RETURN_RESULT;
  }
  Result<Source> createCosineSource(SampleType sampleType, float sampleRate, float frequency,
                                    ICudaCommandQueue* queue) noexcept final {
    if (sampleType == SampleType_FloatComplex) return CosineSource::create(true, sampleRate, frequency, queue, mF);
    if (sampleType == SampleType_Float) return CosineSource::create(false, sampleRate, frequency, queue, mF);
    gsloge("Sample type [%u] is not supported for cosine", sampleType);
    return ERR_RESULT(Status_InvalidArgument);
  }

 private:
  IFactories* const mF;
  REF_COUNTED(CosineSourceFactory);
};

class MemcpyFilterFactory final : public ICudaMemcpyFilterFactory {
 public:
  explicit MemcpyFilterFactory(IFactories* f) noexcept : mF(f) {}
  Result<Node> create(const char* jsonParameters) noexcept final {
    try {
      Json p;
      if (!parseParams(jsonParameters, p)) return ERR_RESULT(Status_ParseError);
      const Json* from = p.get("from");
      const Json* to = p.get("to");
      auto side = [](const Json* j, bool& host) {
        if (j == nullptr || !j->isString()) return false;
        if (j->string() == "host") host = true;
        else if (j->string() == "device") host = false;
        else return false;
        return true;
      };
      bool fromHost = false, toHost = false;
      if (!side(from, fromHost) || !side(to, toHost)) {
        gsloge("HIP memcpy node needs \"from\" and \"to\" in {host, device}");
        return ERR_RESULT(Status_ParseError);
      }
      const hipMemcpyKind kind = fromHost ? (toHost ? hipMemcpyHostToHost : hipMemcpyHostToDevice)
                                          : (toHost ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice);
      Ref<ICudaCommandQueue> q;
      UNWRAP_OR_FWD_RESULT(q, queueFromParams(mF, p));
      return ResultCast<Node>(createCudaMemcpy(kind, q.get().get()));
    }
    IF_CATCH_RETURN_RESULT;
  }
  Result<Filter> createCudaMemcpy(hipMemcpyKind kind, ICudaCommandQueue* queue) noexcept final {
    return HipMemcpyFilter::create(kind, queue, mF);
  }

 private:
  IFactories* const mF;
  REF_COUNTED(MemcpyFilterFactory);
};

// ---- host egress sink (MI355X extension: the AAC writer's D2H + wait-previous path without the codec) ----
class HostSinkFactory final : public INodeFactory {
 public:
  explicit HostSinkFactory(IFactories* f) noexcept : mF(f) {}
  Result<Node> create(const char* jsonParameters) noexcept final {
    try {
      Json p;
      if (!parseParams(jsonParameters, p)) return ERR_RESULT(Status_ParseError);
      Ref<ICudaCommandQueue> q;
      UNWRAP_OR_FWD_RESULT(q, queueFromParams(mF, p));
      return ResultCast<Node>(HostEgressSink::create(q.get().get(), mF));
    }
    IF_CATCH_RETURN_RESULT;
  }

 private:
  IFactories* const mF;
  REF_COUNTED(HostSinkFactory);
};

// ---- device sink (MI355X extension: the end of a chain whose output stays in HBM) ------------------------
class DeviceSinkFactory final : public INodeFactory {
 public:
  explicit DeviceSinkFactory(IFactories* f) noexcept : mF(f) {}
  Result<Node> create(const char* jsonParameters) noexcept final {
    try {
      Json p;
      if (!parseParams(jsonParameters, p)) return ERR_RESULT(Status_ParseError);
      Ref<ICudaCommandQueue> q;
      UNWRAP_OR_FWD_RESULT(q, queueFromParams(mF, p));
      const Json* pb = p.get("preferredBytes");  // optional; 0 / absent: the device-node default
      const size_t preferred = pb != nullptr && pb->isNumber() && pb->number() > 0 ? (size_t)pb->number() : 0;
      return ResultCast<Node>(DeviceSink::create(preferred, q.get().get(), mF));
    }
    IF_CATCH_RETURN_RESULT;
  }

 private:
  IFactories* const mF;
  REF_COUNTED(DeviceSinkFactory);
};

// ---- out-of-scope factories: valid objects whose creators report Status_NotFound ----------------------------
#define GS_OUT_OF_SCOPE(what__)            \
  do {                                     \
    gsloge("%s %s", what__, kOutOfScope);  \
    return ERR_RESULT(Status_NotFound);    \
  } while (false)

class StubAacWriterFactory final : public IAacFileWriterFactory {
 public:
  Result<Node> create(const char*) noexcept final { GS_OUT_OF_SCOPE("AacWriter"); }
  Result<Sink> createAacFileWriter(const char*, int32_t, int32_t, ICudaCommandQueue*) noexcept final {
    GS_OUT_OF_SCOPE("AacWriter");
  }
  REF_COUNTED(StubAacWriterFactory);
};
class StubAddConstFactory final : public IAddConstFactory {
 public:
  Result<Node> create(const char*) noexcept final { GS_OUT_OF_SCOPE("AddConst"); }
  Result<Filter> createAddConst(float, ICudaCommandQueue*) noexcept final { GS_OUT_OF_SCOPE("AddConst"); }
  REF_COUNTED(StubAddConstFactory);
};
class StubAddConstToVectorLengthFactory final : public IAddConstToVectorLengthFactory {
 public:
  Result<Node> create(const char*) noexcept final { GS_OUT_OF_SCOPE("AddConstToVectorLength"); }
  Result<Filter> createAddConstToVectorLength(float, ICudaCommandQueue*) noexcept final {
    GS_OUT_OF_SCOPE("AddConstToVectorLength");
  }
  REF_COUNTED(StubAddConstToVectorLengthFactory);
};
class StubFileReaderFactory final : public IFileReaderFactory {
 public:
  Result<Node> create(const char*) noexcept final { GS_OUT_OF_SCOPE("File"); }
  Result<Source> createFileReader(const char*) noexcept final { GS_OUT_OF_SCOPE("File"); }
  REF_COUNTED(StubFileReaderFactory);
};
class StubHackrfFactory final : public IHackrfSourceFactory {
 public:
  Result<Node> create(const char*) noexcept final { GS_OUT_OF_SCOPE("HackRfSource"); }
  Result<IHackrfSource> createHackrfSource(int32_t, uint64_t, double, size_t) noexcept final {
    GS_OUT_OF_SCOPE("HackRfSource");
  }
  REF_COUNTED(StubHackrfFactory);
};
class StubQueueFilterFactory final : public ICudaFilterFactory {
 public:
  explicit StubQueueFilterFactory(const char* name) noexcept : mName(name) {}
  Result<Node> create(const char*) noexcept final { GS_OUT_OF_SCOPE(mName); }
  Result<Filter> createFilter(ICudaCommandQueue*) noexcept final { GS_OUT_OF_SCOPE(mName); }

 private:
  const char* mName;
  REF_COUNTED(StubQueueFilterFactory);
};
class StubDriverToDotFactory final : public IDriverToDiagramFactory {
 public:
  Result<IDriverToDiagram> create() const noexcept final { GS_OUT_OF_SCOPE("DriverToDot"); }
  REF_COUNTED(StubDriverToDotFactory);
};

// ---- the singleton -----------------------------------------------------------------------------------------
class Factories final : public IFactories {
 public:
  Factories()
      : mRanges(new BufferRangeFactory()),
        mSysAlloc(new SysMemAllocator()),
        mSysCopier(new SysMemCopier()),
        mSysMemSet(new SysMemSet()),
        mHipAllocs(new HipAllocatorFactory()),
        mHipCopiers(new HipCopierFactory()),
        mHipMemSets(new HipMemSetFactory()),
        mResizable(new ResizableBufferFactory(mSysAlloc, mSysCopier, mRanges)),
        mSlices(new BufferSliceFactory(mRanges)),
        mBufferUtil(new BufferUtil()),
        mHipQueues(new HipCommandQueueFactory()),
        mNamedQueues(new CommandQueueFactory(mHipQueues)),
        mMemcpy(new MemcpyFilterFactory(this)),
        mFir(new FirFactory(this)),
        mQuadDemod(new QuadDemodFactory(this)),
        mInt8ToFloat(new QueueFilterFactory(this, &Int8ToFloat::create)),
        mMagnitude(new QueueFilterFactory(this, &QuadAmDemod::create)),
        mCosine(new CosineSourceFactory(this)),
        mAac(new StubAacWriterFactory()),
        mAddConst(new StubAddConstFactory()),
        mAddConstLen(new StubAddConstToVectorLengthFactory()),
        mFile(new StubFileReaderFactory()),
        mHackrf(new StubHackrfFactory()),
        mMultiply(new QueueFilterFactory(this, &MultiplyCcc::create)),
        mStepping(new SteppingDriverFactory()),
        mComponent(newFilterDriverFactory(this)),
        mRemapSink(newPortRemappingSinkFactory()),
        mRemapSource(newPortRemappingSourceFactory()),
        mRfToPcm(newRfToPcmAudioFactory(this)),
        mMonitor(newReadByteCountMonitorFactory()),
        mDot(new StubDriverToDotFactory()) {}

  IResizableBufferFactory* getResizableBufferFactory() noexcept final { return mResizable; }
  ICudaAllocatorFactory* getCudaAllocatorFactory() noexcept final { return mHipAllocs; }
  IBufferSliceFactory* getBufferSliceFactory() noexcept final { return mSlices; }
  IAllocator* getSysMemAllocator() noexcept final { return mSysAlloc; }
  IBufferCopier* getSysMemCopier() noexcept final { return mSysCopier; }
  ICudaBufferCopierFactory* getCudaBufferCopierFactory() noexcept final { return mHipCopiers; }
  IBufferUtil* getBufferUtil() noexcept final { return mBufferUtil; }
  ICudaMemcpyFilterFactory* getCudaMemcpyFilterFactory() noexcept final { return mMemcpy; }
  IAacFileWriterFactory* getAacFileWriterFactory() noexcept final { return mAac; }
  IAddConstFactory* getAddConstFactory() noexcept final { return mAddConst; }
  IAddConstToVectorLengthFactory* getAddConstToVectorLengthFactory() noexcept final { return mAddConstLen; }
  ICosineSourceFactory* getCosineSourceFactory() noexcept final { return mCosine; }
  IFileReaderFactory* getFileReaderFactory() noexcept final { return mFile; }
  IFirFactory* getFirFactory() noexcept final { return mFir; }
  IHackrfSourceFactory* getHackrfSourceFactory() noexcept final { return mHackrf; }
  ICudaFilterFactory* getInt8ToFloatFactory() noexcept final { return mInt8ToFloat; }
  ICudaFilterFactory* getMagnitudeFactory() noexcept final { return mMagnitude; }
  ICudaFilterFactory* getMultiplyFactory() noexcept final { return mMultiply; }
  IQuadDemodFactory* getQuadDemodFactory() noexcept final { return mQuadDemod; }
  IMemSet* getSysMemSet() noexcept final { return mSysMemSet; }
  ICudaMemSetFactory* getCudaMemSetFactory() noexcept final { return mHipMemSets; }
  ISteppingDriverFactory* getSteppingDriverFactory() noexcept final { return mStepping; }
  IFilterDriverFactory* getFilterDriverFactory() noexcept final { return mComponent; }
  IPortRemappingSinkFactory* getPortRemappingSinkFactory() noexcept final { return mRemapSink; }
  IPortRemappingSourceFactory* getPortRemappingSourceFactory() noexcept final { return mRemapSource; }
  IRfToPcmAudioFactory* getRfToPcmAudioFactory() noexcept final { return mRfToPcm; }
  IReadByteCountMonitorFactory* getReadByteCountMonitorFactory() noexcept final { return mMonitor; }
  IDriverToDiagramFactory* getDriverToDotFactory() noexcept final { return mDot; }
  IBufferRangeFactory* getBufferRangeFactory() noexcept final { return mRanges; }
  ICommandQueueFactory* getCommandQueueFactory() noexcept final { return mNamedQueues; }
  ICudaCommandQueueFactory* getCudaCommandQueueFactory() noexcept final { return mHipQueues; }

  Result<IBufferFactory> createBufferFactory(IAllocator* allocator) noexcept final {
    NON_NULL_PARAM_OR_RET(allocator);
    return makeRefResultNonNull<IBufferFactory>(new (std::nothrow) BufferFactory(allocator, mRanges));
  }
  Result<IRelocatableResizableBufferFactory> createRelocatableResizableBufferFactory(
      IAllocator* allocator, const IBufferCopier* copier) noexcept final {
    NON_NULL_PARAM_OR_RET(allocator);
    NON_NULL_PARAM_OR_RET(copier);
    return makeRefResultNonNull<IRelocatableResizableBufferFactory>(
        new (std::nothrow) RelocatableResizableBufferFactory(allocator, copier, mRanges));
  }
  Result<IBufferPool> createBufferPool(size_t maxBufferCount, size_t bufferSize,
                                       IBufferFactory* bufferFactory) noexcept final {
    NON_NULL_PARAM_OR_RET(bufferFactory);
    return makeRefResultNonNull<IBufferPool>(new (std::nothrow) BufferPool(maxBufferCount, bufferSize, bufferFactory));
  }
  Result<IBufferPoolFactory> createBufferPoolFactory(size_t maxBufferCount,
                                                     IBufferFactory* bufferFactory) noexcept final {
    NON_NULL_PARAM_OR_RET(bufferFactory);
    return makeRefResultNonNull<IBufferPoolFactory>(new (std::nothrow)
                                                        BufferPoolFactory(maxBufferCount, bufferFactory));
  }
  // Host-side (pinned) windows relocate with hipMemcpyDefault: a device-to-device kind on host
  // pointers is not what the reference meant (Factories.h:99-110).
  Result<IRelocatableResizableBufferFactory> createRelocatableCudaBufferFactory(ICudaCommandQueue* queue,
                                                                               size_t alignment,
                                                                               bool useHostMemory) noexcept final {
    Ref<IAllocator> allocator;
    Ref<IBufferCopier> copier;
    UNWRAP_OR_FWD_RESULT(allocator, mHipAllocs->createCudaAllocator(queue, alignment, useHostMemory));
    UNWRAP_OR_FWD_RESULT(copier, mHipCopiers->createBufferCopier(queue, useHostMemory ? hipMemcpyDefault
                                                                                      : hipMemcpyDeviceToDevice));
    return createRelocatableResizableBufferFactory(allocator.get().get(), copier.get().get());
  }

  void ref() const noexcept final {}    // immortal singleton (Factories.cpp:188-191)
  void unref() const noexcept final {}

 private:
  ~Factories() final = default;
  ConstRef<IBufferRangeFactory> mRanges;
  ConstRef<IAllocator> mSysAlloc;
  ConstRef<IBufferCopier> mSysCopier;
  ConstRef<IMemSet> mSysMemSet;
  ConstRef<ICudaAllocatorFactory> mHipAllocs;
  ConstRef<ICudaBufferCopierFactory> mHipCopiers;
  ConstRef<ICudaMemSetFactory> mHipMemSets;
  ConstRef<IResizableBufferFactory> mResizable;
  ConstRef<IBufferSliceFactory> mSlices;
  ConstRef<IBufferUtil> mBufferUtil;
  ConstRef<ICudaCommandQueueFactory> mHipQueues;
  ConstRef<ICommandQueueFactory> mNamedQueues;
  ConstRef<ICudaMemcpyFilterFactory> mMemcpy;
  ConstRef<IFirFactory> mFir;
  ConstRef<IQuadDemodFactory> mQuadDemod;
  ConstRef<ICudaFilterFactory> mInt8ToFloat;
  ConstRef<ICudaFilterFactory> mMagnitude;
  ConstRef<ICosineSourceFactory> mCosine;
  ConstRef<IAacFileWriterFactory> mAac;
  ConstRef<IAddConstFactory> mAddConst;
  ConstRef<IAddConstToVectorLengthFactory> mAddConstLen;
  ConstRef<IFileReaderFactory> mFile;
  ConstRef<IHackrfSourceFactory> mHackrf;
  ConstRef<ICudaFilterFactory> mMultiply;
  ConstRef<ISteppingDriverFactory> mStepping;
  ConstRef<IFilterDriverFactory> mComponent;
  ConstRef<IPortRemappingSinkFactory> mRemapSink;
  ConstRef<IPortRemappingSourceFactory> mRemapSource;
  ConstRef<IRfToPcmAudioFactory> mRfToPcm;
  ConstRef<IReadByteCountMonitorFactory> mMonitor;
  ConstRef<IDriverToDiagramFactory> mDot;
};

}  // namespace gsdr_rt

using namespace gsdr_rt;

GS_EXPORT Result<IFactories> getFactoriesSingleton() noexcept {
  static std::once_flag once;
  static Factories* instance = nullptr;  // immortal: never destroyed
  try {
    std::call_once(once, []() { instance = new (std::nothrow) Factories(); });
  }
  IF_CATCH_RETURN_RESULT;
  return makeRefResultNonNull<IFactories>(instance);
}

// ---- node registry (FilterFactories.cpp:23-150) ----------------------------------------------------------
namespace {
std::mutex gRegistryLock;
std::unordered_map<std::string, ImmutableRef<INodeFactory>>& registry() {
  static auto* m = new std::unordered_map<std::string, ImmutableRef<INodeFactory>>();
  return *m;
}

const char* kindString(Node* n) {
  static thread_local std::string s;
  s = std::string("Source? [") + (n->asSource() ? "yes" : "no") + "] Sink? [" + (n->asSink() ? "yes" : "no") +
      "] Filter? [" + (n->asFilter() ? "yes" : "no") + "] Component? [" + (n->asDriver() ? "yes" : "no") + "]";
  return s.c_str();
}
}  // namespace

GS_EXPORT Result<Node> createNode(const char* name, const char* jsonParameters) noexcept {
  try {
    if (name == nullptr) return ERR_RESULT(Status_InvalidArgument);
    Ref<INodeFactory> factory;
    {
      std::lock_guard<std::mutex> l(gRegistryLock);
      auto it = registry().find(name);
      if (it == registry().end()) {
        gsloge("No node factory is registered for [%s]", name);
        return ERR_RESULT(Status_NotFound);
      }
      factory = it->second.get();
    }
    return factory->create(jsonParameters);
  }
  IF_CATCH_RETURN_RESULT;
}

// The new node is floating (ref-count 0) and must be handed on floating: holding it in a Ref
// here would delete it when the Ref goes out of scope. (The reference wraps it in Ref +
// ConstRef and returns the raw pointer, FilterFactories.cpp:44-65, which leaves the caller a
// dangling pointer.)
template <typename T>
static Result<T> createAs(const char* name, const char* json, T* (Node::*as)() noexcept, const char* what) noexcept {
  RefResult<Node> created = createNode(name, json);
  if (created.status != Status_Success) {
    if (created.value != nullptr) created.value->unref();
    return ERR_RESULT(created.status);
  }
  Node* node = created.value;
  T* typed = (node->*as)();
  if (typed == nullptr) {
    gsloge("[%s] was created, but is not a %s. %s", name, what, kindString(node));
    node->unref();  // floating: unref at count 0 deletes
    return ERR_RESULT(Status_InvalidArgument);
  }
  return makeRefResultNonNull<T>(typed);
}

GS_EXPORT Result<Filter> createFilter(const char* name, const char* jsonParameters) noexcept {
  return createAs<Filter>(name, jsonParameters, &Node::asFilter, "Filter");
}
GS_EXPORT Result<Source> createSource(const char* name, const char* jsonParameters) noexcept {
  return createAs<Source>(name, jsonParameters, &Node::asSource, "Source");
}
GS_EXPORT Result<Sink> createSink(const char* name, const char* jsonParameters) noexcept {
  return createAs<Sink>(name, jsonParameters, &Node::asSink, "Sink");
}

GS_EXPORT bool hasNodeFactory(const char* name) noexcept {
  try {
    std::lock_guard<std::mutex> l(gRegistryLock);
    return name != nullptr && registry().count(name) != 0;
  } catch (...) {
    return false;
  }
}

GS_EXPORT Status registerNodeFactory(const char* name, INodeFactory* factory) noexcept {
  try {
    if (name == nullptr) return Status_InvalidArgument;
    std::lock_guard<std::mutex> l(gRegistryLock);
    registry().erase(name);
    if (factory != nullptr) registry().emplace(name, ImmutableRef<INodeFactory>(factory));
    return Status_Success;
  }
  IF_CATCH_RETURN_STATUS;
}

GS_EXPORT Status registerDefaultNodeFactories() noexcept {
  Ref<IFactories> f;
  UNWRAP_OR_FWD_STATUS(f, getFactoriesSingleton());
  IFactories* F = f.get().get();
  FWD_IF_ERR(registerNodeFactory("AacWriter", F->getAacFileWriterFactory()));
  FWD_IF_ERR(registerNodeFactory("AddConst", F->getAddConstFactory()));
  FWD_IF_ERR(registerNodeFactory("AddConstToVectorLength", F->getAddConstToVectorLengthFactory()));
  FWD_IF_ERR(registerNodeFactory("Component", F->getFilterDriverFactory()));
  FWD_IF_ERR(registerNodeFactory("Cosine", F->getCosineSourceFactory()));
  FWD_IF_ERR(registerNodeFactory("File", F->getFileReaderFactory()));
  FWD_IF_ERR(registerNodeFactory("Fir", F->getFirFactory()));
  FWD_IF_ERR(registerNodeFactory("HackRfSource", F->getHackrfSourceFactory()));
  FWD_IF_ERR(registerNodeFactory("Int8ToFloat", F->getInt8ToFloatFactory()));
  FWD_IF_ERR(registerNodeFactory("Magnitude", F->getMagnitudeFactory()));
  FWD_IF_ERR(registerNodeFactory("MultiplyCCC", F->getMultiplyFactory()));
  FWD_IF_ERR(registerNodeFactory("QuadDemod", F->getQuadDemodFactory()));
  FWD_IF_ERR(registerNodeFactory("HipMemcpy", F->getCudaMemcpyFilterFactory()));
  // extension: the host egress sink (D2H end of a chain, one step in flight)
  {
    Ref<INodeFactory> hostSink(new (std::nothrow) HostSinkFactory(F));
    if (hostSink == nullptr) return Status_OutOfMemory;
    FWD_IF_ERR(registerNodeFactory("HostSink", hostSink.get().get()));
  }
  {
    Ref<INodeFactory> deviceSink(new (std::nothrow) DeviceSinkFactory(F));
    if (deviceSink == nullptr) return Status_OutOfMemory;
    FWD_IF_ERR(registerNodeFactory("DeviceSink", deviceSink.get().get()));
  }
  // extension: the RF -> PCM component by name (the reference only reaches it through IFactories)
  FWD_IF_ERR(registerNodeFactory("RfToPcmAudio", F->getRfToPcmAudioFactory()));
  return Status_Success;
}

GS_EXPORT Status registerDefaultFilterFactories() noexcept { return registerDefaultNodeFactories(); }
