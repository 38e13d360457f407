// Time-sharded stream executor (include/gsdr/gsdr_amd.h, gsdrShardStream*): the per-rank step of
// gpusdr/shard.py's HaloRing protocol for native callers.
//
//   buf = [ halo (H = T - 1 samples) | segment (L samples) ]          one per rank, fixed address
//   step:  event segReady on `stream`; xstream waits for it
//          exchange(tail = segment[L - H, L) -> next rank, halo <- previous rank) on xstream
//          bulk:  outputs [head, L/D) over segment + (head D - H)        on `stream`
//          rank 0: head outputs [0, head) over buf (the halo that arrived last step), then
//                  `stream` waits for the exchange and copies incoming -> halo for the next step
//          rank > 0: `stream` waits for the exchange, then the head launch
// At one rank: a single launch over buf, then the tail is copied into the halo; or, with an exchange
// hook, the ring protocol on a ring of one (rank 0's path, the tail sent to itself).
// The FIR is the reference count rule over [halo | segment] (Fir.cpp:178-186): H + L inputs give
// exactly L / D outputs because L % D == 0.
#include <gsdr/gsdr_amd.h>
#include <gpusdrpipeline/GSLog.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <mutex>
#include <new>

namespace {

#define SHS_TRY(expr__)                \
  do {                                 \
    const hipError_t e__ = (expr__);   \
    if (e__ != hipSuccess) return e__; \
  } while (false)

struct DevicePush {
  int prev = -1;
  bool ok = true;
  explicit DevicePush(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DevicePush() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// librccl, loaded on first use so the library itself does not depend on it
struct Rccl {
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGetUniqueId) getUniqueId = nullptr;
  decltype(&ncclCommInitRank) commInitRank = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  bool ok = false;
};

// The calling thread's last RCCL result (gsdrShardRcclLastResult).
thread_local ncclResult_t tLastResult = ncclSuccess;

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) return;
    r.groupStart = reinterpret_cast<decltype(&ncclGroupStart)>(dlsym(h, "ncclGroupStart"));
    r.groupEnd = reinterpret_cast<decltype(&ncclGroupEnd)>(dlsym(h, "ncclGroupEnd"));
    r.send = reinterpret_cast<decltype(&ncclSend)>(dlsym(h, "ncclSend"));
    r.recv = reinterpret_cast<decltype(&ncclRecv)>(dlsym(h, "ncclRecv"));
    r.getUniqueId = reinterpret_cast<decltype(&ncclGetUniqueId)>(dlsym(h, "ncclGetUniqueId"));
    r.commInitRank = reinterpret_cast<decltype(&ncclCommInitRank)>(dlsym(h, "ncclCommInitRank"));
    r.commDestroy = reinterpret_cast<decltype(&ncclCommDestroy)>(dlsym(h, "ncclCommDestroy"));
    r.errorString = reinterpret_cast<decltype(&ncclGetErrorString)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.groupStart && r.groupEnd && r.send && r.recv && r.getUniqueId && r.commInitRank && r.commDestroy &&
           r.errorString;
  });
  return r;
}

// Record an RCCL result for the calling thread; a failure is logged with RCCL's text and the call
// that made it, and becomes hipErrorUnknown for the hipError_t-returning entry points.
hipError_t ncclStatus(const Rccl& r, ncclResult_t res, const char* what) {
  tLastResult = res;
  if (res == ncclSuccess) return hipSuccess;
  gsloge("%s failed: ncclResult_t %d (%s)", what, (int)res, r.errorString ? r.errorString(res) : "?");
  return hipErrorUnknown;
}

}  // namespace

struct gsdrShardStreamImpl {
  int32_t device = 0, rank = 0, world = 1;
  bool int8Iq = false, am = true;
  size_t T = 0, D = 1, L = 0, H = 0;
  size_t elem = 8;      // input bytes per sample
  size_t outElem = 4;   // output bytes per output
  size_t outputs = 0, head = 0, bulkOffset = 0;
  float* taps = nullptr;
  uint8_t* buf = nullptr;
  uint8_t* incoming = nullptr;
  hipStream_t xstream = nullptr;
  hipEvent_t segReady = nullptr, exchanged = nullptr;
  hipEvent_t stepDone = nullptr;  // the last step's completion on its stream (Destroy waits for it)
  bool stepped = false;      // stepDone marks the end of the last enqueued step
  bool syncDevice = false;   // a failed step's end could not be recorded: destroy synchronises the device
  bool ring = false;              // the ring protocol (world > 1, or a ring of one with a hook)
  gsdrHaloExchangeFn exchange = nullptr;
  void* user = nullptr;

  hipError_t fir(const uint8_t* in, size_t n, uint8_t* out, hipStream_t stream) const {
    if (n == 0) return hipSuccess;
    if (int8Iq) {
      const auto* x = reinterpret_cast<const int8_t*>(in);
      return am ? gsdrInt8FirFCAmDemod(D, taps, T, x, reinterpret_cast<float*>(out), n, device, stream)
                : gsdrInt8FirFC(D, taps, T, x, reinterpret_cast<hipFloatComplex*>(out), n, device, stream);
    }
    const auto* x = reinterpret_cast<const hipFloatComplex*>(in);
    return am ? gsdrFirFCAmDemod(D, taps, T, x, reinterpret_cast<float*>(out), n, device, stream)
              : gsdrFirFC(D, taps, T, x, reinterpret_cast<hipFloatComplex*>(out), n, device, stream);
  }

  void release() {
    DevicePush push(device);
    if (segReady) (void)hipEventDestroy(segReady);
    if (stepDone) (void)hipEventDestroy(stepDone);
    if (exchanged) (void)hipEventDestroy(exchanged);
    if (xstream) (void)hipStreamDestroy(xstream);
    (void)hipFree(taps);
    (void)hipFree(buf);
    (void)hipFree(incoming);
  }
};

extern "C" {

GSDR_API hipError_t gsdrShardStreamCreate(int32_t rank, int32_t world, int32_t int8Iq, int32_t am, const float* taps,
                                          size_t tapCount, size_t decimation, size_t segmentSamples,
                                          gsdrHaloExchangeFn exchange, void* user, int32_t device,
                                          gsdrShardStream* streamOut) {
  if (streamOut == nullptr) return hipErrorInvalidValue;
  *streamOut = nullptr;
  if (taps == nullptr || tapCount == 0 || decimation == 0 || world < 1 || rank < 0 || rank >= world)
    return hipErrorInvalidValue;
  if (segmentSamples % decimation != 0 || segmentSamples < tapCount - 1 || segmentSamples == 0)
    return hipErrorInvalidValue;
  if (world > 1 && exchange == nullptr) return hipErrorInvalidValue;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  auto* s = new (std::nothrow) gsdrShardStreamImpl();
  if (s == nullptr) return hipErrorOutOfMemory;
  s->device = device;
  s->rank = rank;
  s->world = world;
  s->int8Iq = int8Iq != 0;
  s->am = am != 0;
  s->T = tapCount;
  s->D = decimation;
  s->L = segmentSamples;
  s->H = tapCount - 1;
  s->elem = s->int8Iq ? 2 : 8;
  s->outElem = s->am ? 4 : 8;
  s->outputs = s->L / s->D;
  s->head = (s->H + s->D - 1) / s->D < s->outputs ? (s->H + s->D - 1) / s->D : s->outputs;  // k D < T - 1
  s->bulkOffset = s->head * s->D - s->H;  // into the segment: the first input of output `head`
  s->exchange = exchange;
  s->user = user;
  s->ring = world > 1 || exchange != nullptr;
  hipError_t e = hipMalloc(&s->taps, tapCount * sizeof(float));
  if (e == hipSuccess) e = hipMemcpy(s->taps, taps, tapCount * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&s->buf, (s->H + s->L) * s->elem);
  if (e == hipSuccess) e = hipMemset(s->buf, 0, (s->H + s->L) * s->elem);
  if (e == hipSuccess && s->ring && rank == 0 && s->H > 0) {
    e = hipMalloc(&s->incoming, s->H * s->elem);
    if (e == hipSuccess) e = hipMemset(s->incoming, 0, s->H * s->elem);
  }
  if (e == hipSuccess && s->ring) e = hipStreamCreateWithFlags(&s->xstream, hipStreamNonBlocking);
  if (e == hipSuccess && s->ring) e = hipEventCreateWithFlags(&s->segReady, hipEventDisableTiming);
  if (e == hipSuccess && s->ring) e = hipEventCreateWithFlags(&s->exchanged, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&s->stepDone, hipEventDisableTiming);
  if (e != hipSuccess) {
    s->release();
    delete s;
    return e;
  }
  *streamOut = s;
  return hipSuccess;
}

GSDR_API void gsdrShardStreamDestroy(gsdrShardStream s) {
  if (s == nullptr) return;
  {
    // no launch or exchange may still use the buffers: the last step's end on its stream (which
    // waited for the exchange) and the exchange stream itself - not the whole device, which would
    // stall every other stream of the application
    DevicePush push(s->device);
    if (s->syncDevice) (void)hipDeviceSynchronize();
    else if (s->stepped) (void)hipEventSynchronize(s->stepDone);
    if (s->xstream) (void)hipStreamSynchronize(s->xstream);
  }
  s->release();
  delete s;
}

GSDR_API void* gsdrShardStreamSegment(gsdrShardStream s) { return s == nullptr ? nullptr : s->buf + s->H * s->elem; }

GSDR_API void* gsdrShardStreamHalo(gsdrShardStream s) { return s == nullptr ? nullptr : s->buf; }

GSDR_API size_t gsdrShardStreamOutputCount(gsdrShardStream s) { return s == nullptr ? 0 : s->outputs; }

// One step's enqueues; the caller records the step's end whatever this returns.
static hipError_t shardStep(gsdrShardStream s, uint8_t* out, hipStream_t stream, bool& enqueued) {
  uint8_t* tail = s->buf + s->L * s->elem;  // segment[L - H, L) = buf[L, L + H)
  const size_t haloBytes = s->H * s->elem;
  enqueued = true;  // from here on work of this step may be queued on `stream` / xstream
  if (!s->ring) {
    SHS_TRY(s->fir(s->buf, s->outputs, out, stream));
    if (haloBytes > 0) SHS_TRY(hipMemcpyAsync(s->buf, tail, haloBytes, hipMemcpyDeviceToDevice, stream));
    return hipSuccess;
  }
  uint8_t* dst = s->rank == 0 ? s->incoming : s->buf;
  const int32_t next = (s->rank + 1) % s->world, prev = (s->rank + s->world - 1) % s->world;
  SHS_TRY(hipEventRecord(s->segReady, stream));
  SHS_TRY(hipStreamWaitEvent(s->xstream, s->segReady, 0));
  if (haloBytes > 0) SHS_TRY(s->exchange(s->user, tail, dst, haloBytes, next, prev, s->xstream));
  SHS_TRY(hipEventRecord(s->exchanged, s->xstream));
  SHS_TRY(s->fir(s->buf + (s->H + s->bulkOffset) * s->elem, s->outputs - s->head, out + s->head * s->outElem, stream));
  if (s->rank == 0) {
    SHS_TRY(s->fir(s->buf, s->head, out, stream));  // the halo that arrived during the previous step
    SHS_TRY(hipStreamWaitEvent(stream, s->exchanged, 0));
    if (haloBytes > 0) SHS_TRY(hipMemcpyAsync(s->buf, s->incoming, haloBytes, hipMemcpyDeviceToDevice, stream));
  } else {
    SHS_TRY(hipStreamWaitEvent(stream, s->exchanged, 0));
    SHS_TRY(s->fir(s->buf, s->head, out, stream));
  }
  return hipSuccess;
}

GSDR_API hipError_t gsdrShardStreamStep(gsdrShardStream s, void* output, hipStream_t stream) {
  if (s == nullptr || output == nullptr) return hipErrorInvalidValue;
  DevicePush push(s->device);
  if (!push.ok) return hipErrorInvalidDevice;
  bool enqueued = false;
  const hipError_t e = shardStep(s, static_cast<uint8_t*>(output), stream, enqueued);
  if (enqueued) {
    // every exit after the first enqueue - a failed launch or exchange included - marks the step's end,
    // so destroy waits for whatever of it was queued. Where even that fails, destroy
    // falls back to a device synchronisation.
    if (s->ring) (void)hipStreamWaitEvent(stream, s->exchanged, 0);
    if (hipEventRecord(s->stepDone, stream) == hipSuccess) s->stepped = true;
    else s->syncDevice = true;
  }
  return e;
}

GSDR_API hipError_t gsdrShardExchangeRccl(void* ncclComm, const void* sendTail, void* recvHalo, size_t bytes,
                                          int32_t nextRank, int32_t prevRank, hipStream_t xstream) {
  const Rccl& r = rccl();
  if (!r.ok) return hipErrorSharedObjectInitFailed;
  auto comm = static_cast<ncclComm_t>(ncclComm);
  SHS_TRY(ncclStatus(r, r.groupStart(), "ncclGroupStart"));
  const ncclResult_t a = r.send(sendTail, bytes, ncclUint8, nextRank, comm, xstream);
  const ncclResult_t b = r.recv(recvHalo, bytes, ncclUint8, prevRank, comm, xstream);
  const ncclResult_t c = r.groupEnd();  // always closes the group, even after a failed send / recv
  SHS_TRY(ncclStatus(r, a, "ncclSend (halo tail)"));
  SHS_TRY(ncclStatus(r, b, "ncclRecv (halo)"));
  return ncclStatus(r, c, "ncclGroupEnd (halo exchange)");
}

GSDR_API hipError_t gsdrShardRcclGetUniqueId(void* uniqueId128) {
  if (uniqueId128 == nullptr) return hipErrorInvalidValue;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  const Rccl& r = rccl();
  if (!r.ok) return hipErrorSharedObjectInitFailed;
  return ncclStatus(r, r.getUniqueId(static_cast<ncclUniqueId*>(uniqueId128)), "ncclGetUniqueId");
}

GSDR_API hipError_t gsdrShardRcclCommCreate(int32_t nranks, const void* uniqueId128, int32_t rank, int32_t device,
                                            void** ncclCommOut) {
  if (ncclCommOut == nullptr || uniqueId128 == nullptr || nranks < 1 || rank < 0 || rank >= nranks)
    return hipErrorInvalidValue;
  *ncclCommOut = nullptr;
  const Rccl& r = rccl();
  if (!r.ok) return hipErrorSharedObjectInitFailed;
  DevicePush push(device);
  if (!push.ok) return hipErrorInvalidDevice;
  ncclUniqueId id;
  __builtin_memcpy(&id, uniqueId128, sizeof(id));
  ncclComm_t comm = nullptr;
  SHS_TRY(ncclStatus(r, r.commInitRank(&comm, nranks, id, rank), "ncclCommInitRank"));
  *ncclCommOut = comm;
  return hipSuccess;
}

GSDR_API hipError_t gsdrShardRcclCommDestroy(void* ncclComm) {
  if (ncclComm == nullptr) return hipSuccess;
  const Rccl& r = rccl();
  if (!r.ok) return hipErrorSharedObjectInitFailed;
  return ncclStatus(r, r.commDestroy(static_cast<ncclComm_t>(ncclComm)), "ncclCommDestroy");
}

GSDR_API int32_t gsdrShardRcclLastResult(const char** message) {
  if (message != nullptr) {
    const Rccl& r = rccl();
    *message = r.errorString ? r.errorString(tLastResult) : "librccl not loaded";
  }
  return (int32_t)tLastResult;
}

}  // extern "C"
