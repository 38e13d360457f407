// Flat C view of the gpusdrpipeline object model (include/gsdr/gpusdr_flat.h).
#include <gsdr/gpusdr_flat.h>

#include <gpusdrpipeline/Factories.h>
#include <gpusdrpipeline/abi/errors.h>

#include <algorithm>
#include <vector>

#include "../runtime/composite.h"
#include "../runtime/driver.h"
#include "../runtime/filters.h"

namespace {

IFactories* factories() {
  static IFactories* f = getFactoriesSingleton().value;
  return f;
}

template <typename T>
T* as(gspHandle h) {
  return h == nullptr ? nullptr : dynamic_cast<T*>(static_cast<IRef*>(h));
}

// Hand a (possibly floating) object to the caller with one reference.
template <typename T>
uint32_t give(RefResult<T>&& r, gspHandle* out) {
  if (out == nullptr) {
    if (r.value != nullptr && r.status == Status_Success) r.value->unref();
    return Status_InvalidArgument;
  }
  *out = nullptr;
  if (r.status != Status_Success) {
    if (r.value != nullptr) r.value->unref();
    return r.status;
  }
  IRef* ref = static_cast<IRef*>(r.value);
  ref->ref();
  *out = ref;
  return Status_Success;
}

uint32_t push(gspHandle node, size_t port, const void* src, size_t bytes, gspHandle queue) {
  Sink* sink = as<Sink>(node);
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (sink == nullptr || q == nullptr || (src == nullptr && bytes != 0)) return Status_InvalidArgument;
  Ref<IBuffer> b;
  UNWRAP_OR_FWD_STATUS(b, sink->requestBuffer(port, bytes));
  if (bytes != 0) {
    HIP_DEV_PUSH_POP_OR_RET_STATUS(q->cudaDevice());
    // the lent window is device memory, or pinned host memory (the H2D staging filter): the copy
    // direction comes from the pointers (unified addressing)
    const hipError_t e = hipMemcpyAsync(b.get()->writePtr(), src, bytes, hipMemcpyDefault, q->cudaStream());
    if (e != hipSuccess) {
      (void)sink->commitBuffer(port, 0);  // cancel the checkout
      return hipErrorToStatus(e);
    }
  }
  return sink->commitBuffer(port, bytes);
}

}  // namespace

extern "C" {

void gspRelease(gspHandle h) {
  if (h != nullptr) static_cast<IRef*>(h)->unref();
}

uint32_t gspQueueCreate(int32_t device, gspHandle* queueOut) {
  return give(factories()->getCudaCommandQueueFactory()->create(device), queueOut);
}

hipStream_t gspQueueStream(gspHandle queue) {
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  return q == nullptr ? nullptr : q->cudaStream();
}

uint32_t gspQueueSync(gspHandle queue) {
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (q == nullptr) return Status_InvalidArgument;
  HIP_DEV_PUSH_POP_OR_RET_STATUS(q->cudaDevice());
  SAFE_HIP_OR_RET_STATUS(hipStreamSynchronize(q->cudaStream()));
  return Status_Success;
}

uint32_t gspFirCreate(uint32_t tapType, uint32_t elementType, size_t decimation, const float* taps, size_t tapCount,
                      gspHandle queue, gspHandle* filterOut) {
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (q == nullptr) return Status_InvalidArgument;
  return give(factories()->getFirFactory()->createFir(tapType, elementType, decimation, taps, tapCount, q), filterOut);
}

uint32_t gspQuadAmDemodCreate(gspHandle queue, gspHandle* filterOut) {
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (q == nullptr) return Status_InvalidArgument;
  return give(factories()->getQuadDemodFactory()->createQuadDemod(Modulation_Am, 0.0f, 0.0f, q), filterOut);
}

uint32_t gspInt8ToFloatCreate(gspHandle queue, gspHandle* filterOut) {
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (q == nullptr) return Status_InvalidArgument;
  return give(factories()->getInt8ToFloatFactory()->createFilter(q), filterOut);
}

uint32_t gspCosineSourceCreate(uint32_t sampleType, float sampleRate, float frequency, gspHandle queue,
                               gspHandle* sourceOut) {
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (q == nullptr) return Status_InvalidArgument;
  return give(factories()->getCosineSourceFactory()->createCosineSource(sampleType, sampleRate, frequency, q),
              sourceOut);
}

uint32_t gspNamedQueueCreate(const char* queueId, const char* json) {
  return factories()->getCommandQueueFactory()->create(queueId, json);
}

uint32_t gspNamedQueueGet(const char* queueId, gspHandle* queueOut) {
  return give(factories()->getCommandQueueFactory()->getCudaCommandQueue(queueId), queueOut);
}

uint32_t gspNodeCreate(const char* name, const char* json, gspHandle* nodeOut) {
  if (!hasNodeFactory("Fir")) {
    const Status st = registerDefaultNodeFactories();
    if (st != Status_Success) return st;
  }
  return give(createNode(name, json), nodeOut);
}

uint32_t gspSinkPushHost(gspHandle node, size_t port, const void* host, size_t bytes, gspHandle queue) {
  return push(node, port, host, bytes, queue);
}

uint32_t gspSinkPushDevice(gspHandle node, size_t port, const void* device, size_t bytes, gspHandle queue) {
  return push(node, port, device, bytes, queue);
}

uint32_t gspSinkPreferredInputSize(gspHandle node, size_t port, size_t* bytesOut) {
  Sink* s = as<Sink>(node);
  if (s == nullptr || bytesOut == nullptr) return Status_InvalidArgument;
  *bytesOut = s->preferredInputBufferSize(port);
  return Status_Success;
}

uint32_t gspSourceOutputSize(gspHandle node, size_t port, size_t* bytesOut, size_t* alignmentOut) {
  Source* s = as<Source>(node);
  if (s == nullptr) return Status_InvalidArgument;
  if (bytesOut) *bytesOut = s->getOutputDataSize(port);
  if (alignmentOut) *alignmentOut = s->getOutputSizeAlignment(port);
  return Status_Success;
}

uint32_t gspSourceRead(gspHandle node, gspHandle* buffers, size_t bufferCount) {
  Source* s = as<Source>(node);
  if (s == nullptr || (buffers == nullptr && bufferCount != 0)) return Status_InvalidArgument;
  try {
    std::vector<IBuffer*> bufs(bufferCount);
    for (size_t i = 0; i < bufferCount; ++i) {
      bufs[i] = as<IBuffer>(buffers[i]);
      if (bufs[i] == nullptr) return Status_InvalidArgument;
    }
    return s->readOutput(bufs.data(), bufferCount);
  }
  IF_CATCH_RETURN_STATUS;
}

uint32_t gspBufferCreate(gspHandle queue, size_t bytes, gspHandle* bufferOut) {
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (q == nullptr) return Status_InvalidArgument;
  Ref<IAllocator> alloc;
  Ref<IBufferFactory> bf;
  UNWRAP_OR_FWD_STATUS(alloc, factories()->getCudaAllocatorFactory()->createCudaAllocator(q, 32, false));
  UNWRAP_OR_FWD_STATUS(bf, factories()->createBufferFactory(alloc.get().get()));
  return give(bf.get()->createBuffer(bytes), bufferOut);
}

uint32_t gspHostBufferCreate(gspHandle queue, size_t bytes, gspHandle* bufferOut) {
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (q == nullptr) return Status_InvalidArgument;
  Ref<IAllocator> alloc;
  Ref<IBufferFactory> bf;
  UNWRAP_OR_FWD_STATUS(alloc, factories()->getCudaAllocatorFactory()->createCudaAllocator(q, 32, true));
  UNWRAP_OR_FWD_STATUS(bf, factories()->createBufferFactory(alloc.get().get()));
  return give(bf.get()->createBuffer(bytes), bufferOut);
}

uint32_t gspDeviceSinkCreate(gspHandle queue, size_t preferredBytes, gspHandle* sinkOut) {
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (q == nullptr) return Status_InvalidArgument;
  return give(gsdr_rt::DeviceSink::create(preferredBytes, q, factories()), sinkOut);
}

uint32_t gspHostSinkCreate(gspHandle queue, gspHandle* sinkOut) {
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (q == nullptr) return Status_InvalidArgument;
  return give(gsdr_rt::HostEgressSink::create(q, factories()), sinkOut);
}

uint32_t gspHostSinkAvailable(gspHandle sink, size_t* bytesOut) {
  auto* s = as<gsdr_rt::HostEgressSink>(sink);
  if (s == nullptr || bytesOut == nullptr) return Status_InvalidArgument;
  *bytesOut = s->available();
  return Status_Success;
}

uint32_t gspHostSinkRead(gspHandle sink, void* dst, size_t capacity, size_t* bytesOut) {
  auto* s = as<gsdr_rt::HostEgressSink>(sink);
  if (s == nullptr || (dst == nullptr && capacity != 0)) return Status_InvalidArgument;
  const size_t n = s->read(dst, capacity);
  if (bytesOut) *bytesOut = n;
  return Status_Success;
}

uint32_t gspHostSinkFlush(gspHandle sink) {
  auto* s = as<gsdr_rt::HostEgressSink>(sink);
  if (s == nullptr) return Status_InvalidArgument;
  return s->flush();
}

uint32_t gspDesignLowPass(double sampleRate, double cutoff, double transitionWidth, double dbAttenuation, float* taps,
                          size_t capacity, size_t* countOut) {
  std::vector<float> t;
  try {
    FWD_IF_ERR(gsdr_rt::designLowPass(sampleRate, cutoff, transitionWidth, dbAttenuation, t));
  } catch (...) {
    return Status_OutOfMemory;
  }
  if (countOut) *countOut = t.size();
  if (taps == nullptr || capacity < t.size()) return taps == nullptr ? Status_Success : Status_OutOfRange;
  std::copy(t.begin(), t.end(), taps);
  return Status_Success;
}

uint32_t gspBufferSlice(gspHandle buffer, size_t start, size_t end, gspHandle* sliceOut) {
  IBuffer* b = as<IBuffer>(buffer);
  if (b == nullptr) return Status_InvalidArgument;
  return give(factories()->getBufferSliceFactory()->slice(b, start, end), sliceOut);
}

uint32_t gspBufferRange(gspHandle buffer, size_t* offset, size_t* endOffset, size_t* capacity) {
  IBuffer* b = as<IBuffer>(buffer);
  if (b == nullptr) return Status_InvalidArgument;
  if (offset) *offset = b->range()->offset();
  if (endOffset) *endOffset = b->range()->endOffset();
  if (capacity) *capacity = b->range()->capacity();
  return Status_Success;
}

uint32_t gspBufferSetRange(gspHandle buffer, size_t offset, size_t endOffset) {
  IBuffer* b = as<IBuffer>(buffer);
  if (b == nullptr) return Status_InvalidArgument;
  return b->range()->setUsedRange(offset, endOffset);
}

void* gspBufferBase(gspHandle buffer) {
  IBuffer* b = as<IBuffer>(buffer);
  return b == nullptr ? nullptr : b->base();
}

uint32_t gspBufferToHost(gspHandle buffer, void* host, size_t bytes, gspHandle queue) {
  IBuffer* b = as<IBuffer>(buffer);
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (b == nullptr || q == nullptr || (host == nullptr && bytes != 0)) return Status_InvalidArgument;
  const size_t n = bytes < b->range()->used() ? bytes : b->range()->used();
  HIP_DEV_PUSH_POP_OR_RET_STATUS(q->cudaDevice());
  if (n != 0) SAFE_HIP_OR_RET_STATUS(hipMemcpyAsync(host, b->readPtr(), n, hipMemcpyDefault, q->cudaStream()));
  SAFE_HIP_OR_RET_STATUS(hipStreamSynchronize(q->cudaStream()));
  return Status_Success;
}


uint32_t gspSteppingDriverCreate(gspHandle* driverOut) {
  return give(factories()->getSteppingDriverFactory()->createSteppingDriver(), driverOut);
}

uint32_t gspDriverConnect(gspHandle driver, gspHandle source, size_t sourcePort, gspHandle sink, size_t sinkPort) {
  IDriver* d = as<IDriver>(driver);
  Source* so = as<Source>(source);
  Sink* si = as<Sink>(sink);
  if (d == nullptr || so == nullptr || si == nullptr) return Status_InvalidArgument;
  return d->connect(so, sourcePort, si, sinkPort);
}

uint32_t gspDriverSetupNode(gspHandle driver, gspHandle node, const char* name) {
  IDriver* d = as<IDriver>(driver);
  Node* n = as<Node>(node);
  if (d == nullptr || n == nullptr) return Status_InvalidArgument;
  return d->setupNode(n, name);
}

uint32_t gspDriverDoFilterGraphed(gspHandle driver, gspHandle queue) {
  auto* d = dynamic_cast<gsdr_rt::SteppingDriver*>(as<IDriver>(driver));
  ICudaCommandQueue* q = as<ICudaCommandQueue>(queue);
  if (d == nullptr || q == nullptr) return Status_InvalidArgument;
  return d->doFilterGraphed(q->cudaStream());
}

uint32_t gspDriverGraphStats(gspHandle driver, size_t* eager, size_t* captured, size_t* replayed) {
  IDriver* any = as<IDriver>(driver);
  auto* d = dynamic_cast<gsdr_rt::SteppingDriver*>(any);
  if (d == nullptr) d = gsdr_rt::componentSteppingDriver(any);  // a JSON Component's inner driver
  if (d == nullptr) return Status_InvalidArgument;
  const auto st = d->graphStats();
  if (eager) *eager = st.eager;
  if (captured) *captured = st.captured;
  if (replayed) *replayed = st.replayed;
  return Status_Success;
}

uint32_t gspDriverGraphDirectReplays(gspHandle driver, size_t* direct) {
  IDriver* any = as<IDriver>(driver);
  auto* d = dynamic_cast<gsdr_rt::SteppingDriver*>(any);
  if (d == nullptr) d = gsdr_rt::componentSteppingDriver(any);
  if (d == nullptr || direct == nullptr) return Status_InvalidArgument;
  *direct = d->graphStats().direct;
  return Status_Success;
}

uint32_t gspDriverSetFuseFirAm(gspHandle driver, int32_t on) {
  auto* d = dynamic_cast<gsdr_rt::SteppingDriver*>(as<IDriver>(driver));
  if (d == nullptr) return Status_InvalidArgument;
  d->setFuseFirAm(on != 0);
  return Status_Success;
}

uint32_t gspDriverFusedSteps(gspHandle driver, size_t* fused) {
  auto* d = dynamic_cast<gsdr_rt::SteppingDriver*>(as<IDriver>(driver));
  if (d == nullptr || fused == nullptr) return Status_InvalidArgument;
  *fused = d->graphStats().fused;
  return Status_Success;
}

uint32_t gspDriverDoFilter(gspHandle driver) {
  ISteppingDriver* d = as<ISteppingDriver>(driver);
  if (d == nullptr) return Status_InvalidArgument;
  return d->doFilter();
}

size_t gspDriverNodeName(gspHandle driver, gspHandle node, char* name, size_t nameBufLen, int32_t* found) {
  IDriver* d = as<IDriver>(driver);
  Node* n = as<Node>(node);
  bool f = false;
  size_t len = 0;
  if (d != nullptr && n != nullptr) len = d->getNodeName(n, name, nameBufLen, &f);
  if (found != nullptr) *found = f ? 1 : 0;
  return len;
}

}  // extern "C"
