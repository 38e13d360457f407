/*
 * gpusdr_flat.h - a flat C view of the gpusdrpipeline object model for foreign-function
 * callers (Python ctypes in tests/ and bench.py; any cgo / JNI / N-API binding).
 *
 * Every handle is an IRef-derived object holding ONE reference owned by the caller; release it
 * with gspRelease(). Functions return a Status (0 = Status_Success, include/gpusdrpipeline
 * abi/core.h) and never throw. Device work is enqueued on the queue's HIP stream; only
 * gspQueueSync() and gspBufferToHost() block.
 *
 * Reference interfaces each call forwards to:
 *   gspQueueCreate           ICudaCommandQueueFactory::create   (ICudaCommandQueueFactory.h:11-16)
 *   gspFirCreate             IFirFactory::createFir             (FilterFactories.h:101-112)
 *   gspQuadAmDemodCreate     IQuadDemodFactory::createQuadDemod (FilterFactories.h:146-157)
 *   gspInt8ToFloatCreate     ICudaFilterFactory::createFilter   (FilterFactories.h:125-130)
 *   gspCosineSourceCreate    ICosineSourceFactory::createCosineSource
 *   gspNodeCreate            createNode (registry, FilterFactories.h:36)
 *   gspSinkPushHost          Sink::requestBuffer + H2D copy + Sink::commitBuffer (Filter.h:40-66)
 *   gspSourceOutputSize      Source::getOutputDataSize / getOutputSizeAlignment (Filter.h:70-87)
 *   gspSourceRead            Source::readOutput (Filter.h:111-121)
 *   gspBuffer*               IBufferFactory / IBufferSliceFactory / IBufferRange
 */
#ifndef GSDR_GPUSDR_FLAT_H
#define GSDR_GPUSDR_FLAT_H

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define GSP_API __attribute__((visibility("default")))
#else
#define GSP_API
#endif

typedef void* gspHandle; /* an IRef-derived object; one caller-owned reference */

GSP_API void gspRelease(gspHandle h);

GSP_API uint32_t gspQueueCreate(int32_t device, gspHandle* queueOut);
GSP_API hipStream_t gspQueueStream(gspHandle queue);
GSP_API uint32_t gspQueueSync(gspHandle queue);

/* sampleType values: 0 FloatComplex, 1 Float, 2 Int8Complex (SampleType.h:20-25). taps is host memory. */
GSP_API uint32_t gspFirCreate(uint32_t tapType, uint32_t elementType, size_t decimation, const float* taps,
                              size_t tapCount, gspHandle queue, gspHandle* filterOut);
GSP_API uint32_t gspQuadAmDemodCreate(gspHandle queue, gspHandle* filterOut);
GSP_API uint32_t gspInt8ToFloatCreate(gspHandle queue, gspHandle* filterOut);
GSP_API uint32_t gspCosineSourceCreate(uint32_t sampleType, float sampleRate, float frequency, gspHandle queue,
                                       gspHandle* sourceOut);
GSP_API uint32_t gspNamedQueueCreate(const char* queueId, const char* json);
/* The queue a JSON node refers to by name (ICommandQueueFactory::getCudaCommandQueue). */
GSP_API uint32_t gspNamedQueueGet(const char* queueId, gspHandle* queueOut);
GSP_API uint32_t gspNodeCreate(const char* name, const char* json, gspHandle* nodeOut);

/* Sink side of a filter node: append host bytes to input port `port`. */
GSP_API uint32_t gspSinkPushHost(gspHandle node, size_t port, const void* host, size_t bytes, gspHandle queue);
/* Sink side: append bytes already on the device (D2D copy on the queue). */
GSP_API uint32_t gspSinkPushDevice(gspHandle node, size_t port, const void* device, size_t bytes, gspHandle queue);
GSP_API uint32_t gspSinkPreferredInputSize(gspHandle node, size_t port, size_t* bytesOut);

GSP_API uint32_t gspSourceOutputSize(gspHandle node, size_t port, size_t* bytesOut, size_t* alignmentOut);
GSP_API uint32_t gspSourceRead(gspHandle node, gspHandle* buffers, size_t bufferCount);

/* Device buffers (32-byte aligned device memory from the queue's stream-ordered pool). */
GSP_API uint32_t gspBufferCreate(gspHandle queue, size_t bytes, gspHandle* bufferOut);
/* Pinned host buffers (hipHostMalloc through the queue's allocator): outputs of the D2H staging
 * filter. gspBufferBase is then a host pointer. */
GSP_API uint32_t gspHostBufferCreate(gspHandle queue, size_t bytes, gspHandle* bufferOut);
/* Host egress sink (JSON type "HostSink"; the D2H end of a chain, reference AacFileWriter.cpp:267-280
 * without the codec, Waiter.cpp:34-50): its input window is pinned host memory the upstream kernel
 * writes into; each commit leaves one step in flight and hands everything before it to a host FIFO.
 * gspHostSinkRead drains up to `capacity` bytes (count in *bytesOut); gspHostSinkFlush waits for the
 * in-flight step and queues it too. */
GSP_API uint32_t gspHostSinkCreate(gspHandle queue, gspHandle* sinkOut);
/* A device sink that retires every committed byte (a chain's consumer in benchmarks, or a tail
 * whose output is not read back); it asks for preferredBytes per step (0: 256 MiB). */
GSP_API uint32_t gspDeviceSinkCreate(gspHandle queue, size_t preferredBytes, gspHandle* sinkOut);
GSP_API uint32_t gspHostSinkAvailable(gspHandle sink, size_t* bytesOut);
GSP_API uint32_t gspHostSinkRead(gspHandle sink, void* dst, size_t capacity, size_t* bytesOut);
GSP_API uint32_t gspHostSinkFlush(gspHandle sink);
GSP_API uint32_t gspBufferSlice(gspHandle buffer, size_t start, size_t end, gspHandle* sliceOut);
GSP_API uint32_t gspBufferRange(gspHandle buffer, size_t* offset, size_t* endOffset, size_t* capacity);
GSP_API uint32_t gspBufferSetRange(gspHandle buffer, size_t offset, size_t endOffset);
GSP_API void* gspBufferBase(gspHandle buffer);
/* Copies the buffer's used bytes (at most `bytes`) to host and synchronises the queue. */
GSP_API uint32_t gspBufferToHost(gspHandle buffer, void* host, size_t bytes, gspHandle queue);

/* The RF -> PCM component's low-pass designer (Kaiser window, runtime/composite.h; the reference's
 * remez is not vendored): writes the taps if `taps` holds `capacity` >= count floats; *countOut =
 * the tap count. taps == nullptr only reports the count. */
GSP_API uint32_t gspDesignLowPass(double sampleRate, double cutoff, double transitionWidth, double dbAttenuation,
                                  float* taps, size_t capacity, size_t* countOut);

/* SteppingDriver (ISteppingDriver, SteppingDriver.cpp:102-366): connect nodes, name them, and
 * pull one step of every graph tail. Handles are nodes from the creators above. */
GSP_API uint32_t gspSteppingDriverCreate(gspHandle* driverOut);
GSP_API uint32_t gspDriverConnect(gspHandle driver, gspHandle source, size_t sourcePort, gspHandle sink,
                                  size_t sinkPort);
GSP_API uint32_t gspDriverSetupNode(gspHandle driver, gspHandle node, const char* name);
GSP_API uint32_t gspDriverDoFilter(gspHandle driver);
/* MI355X extension: one doFilter step whose device work is replayed from a hipGraph captured per
 * repeating chain state (every node a hot-path filter on `queue`'s stream; otherwise a plain step).
 * gspDriverGraphStats counts plain, capturing and replayed steps. */
GSP_API uint32_t gspDriverDoFilterGraphed(gspHandle driver, gspHandle queue);
GSP_API uint32_t gspDriverGraphStats(gspHandle driver, size_t* eager, size_t* captured, size_t* replayed);
/* Of the replayed steps: those replayed as direct kernel launches (the captured graph was a linear chain
 * of kernel nodes); the rest went through hipGraphLaunch. */
GSP_API uint32_t gspDriverGraphDirectReplays(gspHandle driver, size_t* direct);
/* Fir -> QuadAmDemod fusion (on by default): a Fir with real taps whose only sink is a QuadAmDemod
 * on the same queue is stepped with it as ONE gsdrFirFCAmDemod launch (the same envelopes within
 * the FIR tolerance: the fused launch covers a different span, which moves the FFT / matrix-core
 * kernels' block boundaries and so the last bits of some outputs).
 * gspDriverFusedSteps counts the fused edge moves. */
GSP_API uint32_t gspDriverSetFuseFirAm(gspHandle driver, int32_t on);
GSP_API uint32_t gspDriverFusedSteps(gspHandle driver, size_t* fused);
/* Name given to `node` by setupNode (this driver or a nested one); *found = 0 if none. Returns the
 * name length; at most nameBufLen bytes are written (NUL-terminated when it fits). */
GSP_API size_t gspDriverNodeName(gspHandle driver, gspHandle node, char* name, size_t nameBufLen, int32_t* found);

#ifdef __cplusplus
}
#endif

#endif /* GSDR_GPUSDR_FLAT_H */
