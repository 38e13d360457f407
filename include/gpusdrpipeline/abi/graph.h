/*
 * gpusdrpipeline filter graph (MI355X build): nodes, the node registry, node factories and the
 * driver interfaces.
 *
 * Vtable-compatible with the reference's filters/Filter.h:30-138, filters/FilterFactories.h:30-184,
 * filters/I{HackrfSource,PortRemappingSink,PortRemappingSource,ReadByteCountMonitor}.h and
 * driver/I*.h. Streaming contract (unchanged):
 *   Sink::requestBuffer(port, n)  lends device memory for at least n bytes of input;
 *   Sink::commitBuffer(port, n)   marks n bytes written;
 *   Source::readOutput(bufs, k)   enqueues the processing on the node's HIP stream, appends to
 *                                 each output buffer (never past its capacity), consumes input,
 *                                 and returns without synchronising.
 */
#ifndef GPUSDRPIPELINE_ABI_GRAPH_H
#define GPUSDRPIPELINE_ABI_GRAPH_H

#include <gpusdrpipeline/abi/buffers.h>
#include <gpusdrpipeline/abi/queue.h>

class Sink;
class Source;
class Filter;
class IDriver;

class Node : public virtual IRef {
 public:
  virtual Sink* asSink() noexcept { return nullptr; }
  virtual Source* asSource() noexcept { return nullptr; }
  virtual Filter* asFilter() noexcept { return nullptr; }
  virtual IDriver* asDriver() noexcept { return nullptr; }
  virtual void updateParameters(const char* jsonParameters) noexcept {}

  ABSTRACT_IREF(Node);
};

class Sink : public virtual Node {
 public:
  [[nodiscard]] virtual Result<IBuffer> requestBuffer(size_t port, size_t byteCount) noexcept = 0;
  [[nodiscard]] virtual Status commitBuffer(size_t port, size_t byteCount) noexcept = 0;
  [[nodiscard]] virtual size_t preferredInputBufferSize(size_t port) noexcept = 0;

  [[nodiscard]] Sink* asSink() noexcept override { return this; }

  ABSTRACT_IREF(Sink);
};

class Source : public virtual Node {
 public:
  [[nodiscard]] virtual size_t getOutputDataSize(size_t port) noexcept = 0;
  [[nodiscard]] virtual size_t getOutputSizeAlignment(size_t port) noexcept = 0;
  [[nodiscard]] virtual IBufferCopier* getOutputCopier(size_t port) noexcept = 0;

  /* getOutputDataSize rounded up to the alignment (down if that would overflow). */
  [[nodiscard]] virtual size_t getAlignedOutputDataSize(size_t port) noexcept {
    const size_t a = getOutputSizeAlignment(port);
    const size_t n = getOutputDataSize(port);
    return n > SIZE_MAX - a + 1 ? n / a * a : (n + a - 1) / a * a;
  }

  [[nodiscard]] virtual Status readOutput(IBuffer** portOutputBuffers, size_t numPorts) noexcept = 0;

  [[nodiscard]] Source* asSource() noexcept override { return this; }

  ABSTRACT_IREF(Source);
};

class Filter : public virtual Sink, public virtual Source {
  ABSTRACT_IREF(Filter);

  Filter* asFilter() noexcept override { return this; }
};

/* ---- node registry --------------------------------------------------------------------------- */
class INodeFactory : public virtual IRef {
 public:
  virtual Result<Node> create(const char* jsonParameters) noexcept = 0;

  ABSTRACT_IREF(INodeFactory);
};

GS_EXPORT [[nodiscard]] Result<Node> createNode(const char* name, const char* jsonParameters) noexcept;
GS_EXPORT [[nodiscard]] Result<Filter> createFilter(const char* name, const char* jsonParameters) noexcept;
GS_EXPORT [[nodiscard]] Result<Source> createSource(const char* name, const char* jsonParameters) noexcept;
GS_EXPORT [[nodiscard]] Result<Sink> createSink(const char* name, const char* jsonParameters) noexcept;
GS_EXPORT [[nodiscard]] bool hasNodeFactory(const char* name) noexcept;
GS_EXPORT [[nodiscard]] Status registerNodeFactory(const char* name, INodeFactory* filterFactory) noexcept;
GS_EXPORT [[nodiscard]] Status registerDefaultNodeFactories() noexcept;
/* The reference declares registerDefaultNodeFactories but defines registerDefaultFilterFactories
 * (FilterFactories.h:43 vs FilterFactories.cpp:132); both names are exported here. */
GS_EXPORT [[nodiscard]] Status registerDefaultFilterFactories() noexcept;

/* ---- special node types ----------------------------------------------------------------------- */
class IHackrfSource : public virtual Source {
 public:
  [[nodiscard]] virtual int32_t getDeviceCount() const noexcept = 0;
  [[nodiscard]] virtual size_t getDeviceSerialNumber(int32_t deviceIndex, char* buffer,
                                                     size_t bufferSize) const noexcept = 0;
  [[nodiscard]] virtual Status selectDeviceByIndex(int32_t deviceIndex) noexcept = 0;
  [[nodiscard]] virtual Status selectDeviceBySerialNumber(const char* serialNumber) noexcept = 0;
  [[nodiscard]] virtual Status releaseDevice() noexcept = 0;
  [[nodiscard]] virtual Status start() noexcept = 0;
  [[nodiscard]] virtual Status stop() noexcept = 0;

  ABSTRACT_IREF(IHackrfSource);
};

class IPortRemappingSink : public virtual Sink {
 public:
  virtual void addPortMapping(size_t outerPort, Sink* innerSink, size_t innerSinkPort) noexcept = 0;

  ABSTRACT_IREF(IPortRemappingSink);
};

class IPortRemappingSource : public virtual Source {
 public:
  virtual void addPortMapping(size_t outerPort, Source* innerSource, size_t innerSourcePort) noexcept = 0;

  ABSTRACT_IREF(IPortRemappingSource);
};

class IReadByteCountMonitor : public Filter {
 public:
  [[nodiscard]] virtual size_t getByteCountRead(size_t port) noexcept = 0;

  ABSTRACT_IREF(IReadByteCountMonitor);
};

/* ---- node factories ---------------------------------------------------------------------------- */
class ICudaMemcpyFilterFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<Filter> createCudaMemcpy(hipMemcpyKind memcpyKind,
                                                        ICudaCommandQueue* commandQueue) noexcept = 0;

  ABSTRACT_IREF(ICudaMemcpyFilterFactory);
};

class IAacFileWriterFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<Sink> createAacFileWriter(const char* outputFileName, int32_t sampleRate,
                                                         int32_t bitRate, ICudaCommandQueue* commandQueue) noexcept = 0;

  ABSTRACT_IREF(IAacFileWriterFactory);
};

class IAddConstFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<Filter> createAddConst(float addValueToAmplitude,
                                                      ICudaCommandQueue* commandQueue) noexcept = 0;

  ABSTRACT_IREF(IAddConstFactory);
};

class IAddConstToVectorLengthFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<Filter> createAddConstToVectorLength(float addValueToMagnitude,
                                                                    ICudaCommandQueue* commandQueue) noexcept = 0;

  ABSTRACT_IREF(IAddConstToVectorLengthFactory);
};

class ICosineSourceFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<Source> createCosineSource(SampleType sampleType, float sampleRate, float frequency,
                                                          ICudaCommandQueue* commandQueue) noexcept = 0;

  ABSTRACT_IREF(ICosineSourceFactory);
};

class IFileReaderFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<Source> createFileReader(const char* fileName) noexcept = 0;

  ABSTRACT_IREF(IFileReaderFactory);
};

/* Complex taps are passed as `tapCount` interleaved {re, im} float pairs. */
class IFirFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<Filter> createFir(SampleType tapType, SampleType elementType, size_t decimation,
                                                 const float* taps, size_t tapCount,
                                                 ICudaCommandQueue* commandQueue) noexcept = 0;

  ABSTRACT_IREF(IFirFactory);
};

class IHackrfSourceFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<IHackrfSource> createHackrfSource(int32_t deviceIndex, uint64_t centerFrequency,
                                                                 double sampleRate,
                                                                 size_t maxBufferCountBeforeDropping) noexcept = 0;

  ABSTRACT_IREF(IHackrfSourceFactory);
};

class ICudaFilterFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<Filter> createFilter(ICudaCommandQueue* commandQueue) noexcept = 0;

  ABSTRACT_IREF(ICudaFilterFactory);
};

class IPortRemappingSinkFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IPortRemappingSink> create() noexcept = 0;

  ABSTRACT_IREF(IPortRemappingSinkFactory);
};

class IPortRemappingSourceFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IPortRemappingSource> create() noexcept = 0;

  ABSTRACT_IREF(IPortRemappingSourceFactory);
};

class IQuadDemodFactory : public INodeFactory {
 public:
  /* fskDeviation is only used for FM. */
  [[nodiscard]] virtual Result<Filter> createQuadDemod(Modulation modulation, float rfSampleRate, float fskDeviation,
                                                       ICudaCommandQueue* commandQueue) noexcept = 0;

  ABSTRACT_IREF(IQuadDemodFactory);
};

class IRfToPcmAudioFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<Filter> createRfToPcm(float rfSampleRate, Modulation modulation, size_t rfLowPassDecim,
                                                     size_t audioLowPassDecim, float centerFrequency,
                                                     float channelFrequency, float channelWidth,
                                                     float fskDeviationIfFm, float rfLowPassDbAttenuation,
                                                     float audioLowPassDbAttenuation,
                                                     const char* commandQueueId) noexcept = 0;

  ABSTRACT_IREF(IRfToPcmAudioFactory);
};

class IReadByteCountMonitorFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IReadByteCountMonitor> create(Filter* monitoredFilter) noexcept = 0;

  ABSTRACT_IREF(IReadByteCountMonitorFactory);
};

/* ---- drivers ----------------------------------------------------------------------------------------- */
class IDriver : public virtual Node {
 public:
  IDriver* asDriver() noexcept override { return this; }

  [[nodiscard]] virtual Status connect(Source* source, size_t sourcePort, Sink* sink, size_t sinkPort) noexcept = 0;
  [[nodiscard]] virtual Status setupNode(Node* node, const char* functionInGraph) noexcept = 0;
  virtual void iterateOverConnections(void* context,
                                      void (*connectionIterator)(IDriver* driver, void* context, Source* source,
                                                                 size_t sourcePort, Sink* sink,
                                                                 size_t sinkPort) noexcept) noexcept = 0;
  virtual void iterateOverNodes(void* context,
                                void (*nodeIterator)(IDriver* driver, void* context, Node* node) noexcept) noexcept = 0;
  virtual void iterateOverNodeAttributes(Node* node, void* context,
                                         void (*nodeAttrIterator)(IDriver* driver, Node* node, void* context,
                                                                  const char* attrName,
                                                                  const char* attrVal) noexcept) noexcept = 0;
  virtual size_t getNodeName(Node* node, char* name, size_t nameBufLen, bool* foundOut) noexcept = 0;

  ABSTRACT_IREF(IDriver);
};

class ISteppingDriver : public IDriver {
 public:
  /* One pull of every graph tail through its upstream chain (SteppingDriver.cpp:193-366). */
  [[nodiscard]] virtual Status doFilter() noexcept = 0;

  ABSTRACT_IREF(ISteppingDriver);
};

class IFilterDriver : public IDriver, public Filter {
 public:
  virtual void setDriverInput(Sink* sink) noexcept = 0;
  virtual void setDriverOutput(Source* source) noexcept = 0;

  ABSTRACT_IREF(IFilterDriver);
};

class IDriverToDiagram : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<size_t> convertToDot(IDriver* driver, const char* name, char* diagramBuffer,
                                                    size_t diagramSize) noexcept = 0;

  ABSTRACT_IREF(IDriverToDiagram);
};

class IDriverToDiagramFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IDriverToDiagram> create() const = 0;

  ABSTRACT_IREF(IDriverToDiagramFactory);
};

class IFilterDriverFactory : public INodeFactory {
 public:
  [[nodiscard]] virtual Result<IFilterDriver> createFilterDriver() noexcept = 0;

  ABSTRACT_IREF(IFilterDriverFactory);
};

class ISteppingDriverFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<ISteppingDriver> createSteppingDriver() noexcept = 0;

  ABSTRACT_IREF(ISteppingDriverFactory);
};

#endif  // GPUSDRPIPELINE_ABI_GRAPH_H
