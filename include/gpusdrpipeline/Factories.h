/*
 * IFactories: the root object of the gpusdrpipeline C++ ABI (MI355X build).
 *
 * Slot order is the reference's (include/gpusdrpipeline/Factories.h:41-117): 31 getters, 4 pure
 * creators, 3 overridable helpers. Getters return borrowed pointers owned by the immortal
 * singleton. Getters for subsystems outside this build's hot-path scope (AAC writer, file
 * reader, HackRF, add-const, magnitude, multiply, component/stepping drivers, port remapping,
 * RF->PCM, byte monitor, DOT export) return objects whose creators fail with Status_NotFound,
 * so the vtable and call sites stay valid (DESIGN.md "Out of scope").
 */
#ifndef GPUSDRPIPELINE_FACTORIES_H
#define GPUSDRPIPELINE_FACTORIES_H

#include <gpusdrpipeline/abi/buffers.h>
#include <gpusdrpipeline/abi/core.h>
#include <gpusdrpipeline/abi/graph.h>
#include <gpusdrpipeline/abi/queue.h>

class IFactories : public virtual IRef {
 public:
  [[nodiscard]] virtual IResizableBufferFactory* getResizableBufferFactory() noexcept = 0;
  [[nodiscard]] virtual ICudaAllocatorFactory* getCudaAllocatorFactory() noexcept = 0;
  [[nodiscard]] virtual IBufferSliceFactory* getBufferSliceFactory() = 0;
  [[nodiscard]] virtual IAllocator* getSysMemAllocator() noexcept = 0;
  [[nodiscard]] virtual IBufferCopier* getSysMemCopier() noexcept = 0;
  [[nodiscard]] virtual ICudaBufferCopierFactory* getCudaBufferCopierFactory() noexcept = 0;
  [[nodiscard]] virtual IBufferUtil* getBufferUtil() noexcept = 0;
  [[nodiscard]] virtual ICudaMemcpyFilterFactory* getCudaMemcpyFilterFactory() noexcept = 0;
  [[nodiscard]] virtual IAacFileWriterFactory* getAacFileWriterFactory() noexcept = 0;
  [[nodiscard]] virtual IAddConstFactory* getAddConstFactory() noexcept = 0;
  [[nodiscard]] virtual IAddConstToVectorLengthFactory* getAddConstToVectorLengthFactory() noexcept = 0;
  [[nodiscard]] virtual ICosineSourceFactory* getCosineSourceFactory() noexcept = 0;
  [[nodiscard]] virtual IFileReaderFactory* getFileReaderFactory() noexcept = 0;
  [[nodiscard]] virtual IFirFactory* getFirFactory() noexcept = 0;
  [[nodiscard]] virtual IHackrfSourceFactory* getHackrfSourceFactory() noexcept = 0;
  [[nodiscard]] virtual ICudaFilterFactory* getInt8ToFloatFactory() noexcept = 0;
  [[nodiscard]] virtual ICudaFilterFactory* getMagnitudeFactory() noexcept = 0;
  [[nodiscard]] virtual ICudaFilterFactory* getMultiplyFactory() noexcept = 0;
  [[nodiscard]] virtual IQuadDemodFactory* getQuadDemodFactory() noexcept = 0;
  [[nodiscard]] virtual IMemSet* getSysMemSet() noexcept = 0;
  [[nodiscard]] virtual ICudaMemSetFactory* getCudaMemSetFactory() noexcept = 0;
  [[nodiscard]] virtual ISteppingDriverFactory* getSteppingDriverFactory() noexcept = 0;
  [[nodiscard]] virtual IFilterDriverFactory* getFilterDriverFactory() noexcept = 0;
  [[nodiscard]] virtual IPortRemappingSinkFactory* getPortRemappingSinkFactory() noexcept = 0;
  [[nodiscard]] virtual IPortRemappingSourceFactory* getPortRemappingSourceFactory() noexcept = 0;
  [[nodiscard]] virtual IRfToPcmAudioFactory* getRfToPcmAudioFactory() noexcept = 0;
  [[nodiscard]] virtual IReadByteCountMonitorFactory* getReadByteCountMonitorFactory() noexcept = 0;
  [[nodiscard]] virtual IDriverToDiagramFactory* getDriverToDotFactory() noexcept = 0;
  [[nodiscard]] virtual IBufferRangeFactory* getBufferRangeFactory() noexcept = 0;
  [[nodiscard]] virtual ICommandQueueFactory* getCommandQueueFactory() noexcept = 0;
  [[nodiscard]] virtual ICudaCommandQueueFactory* getCudaCommandQueueFactory() noexcept = 0;

  [[nodiscard]] virtual Result<IBufferFactory> createBufferFactory(IAllocator* allocator) noexcept = 0;
  [[nodiscard]] virtual Result<IRelocatableResizableBufferFactory> createRelocatableResizableBufferFactory(
      IAllocator* allocator, const IBufferCopier* bufferCopier) noexcept = 0;
  [[nodiscard]] virtual Result<IBufferPool> createBufferPool(size_t maxBufferCount, size_t bufferSize,
                                                             IBufferFactory* bufferFactory) noexcept = 0;
  [[nodiscard]] virtual Result<IBufferPoolFactory> createBufferPoolFactory(size_t maxBufferCount,
                                                                           IBufferFactory* bufferFactory) noexcept = 0;

  [[nodiscard]] virtual Result<IRelocatableResizableBufferFactory> createRelocatableSysMemBufferFactory() noexcept {
    return createRelocatableResizableBufferFactory(getSysMemAllocator(), getSysMemCopier());
  }

  [[nodiscard]] virtual Result<IRelocatableResizableBufferFactory> createRelocatableCudaBufferFactory(
      ICudaCommandQueue* commandQueue, size_t cudaAlignment, bool useHostMemory) noexcept {
    Ref<IAllocator> allocator;
    Ref<IBufferCopier> copier;
    UNWRAP_OR_FWD_RESULT(allocator,
                         getCudaAllocatorFactory()->createCudaAllocator(commandQueue, cudaAlignment, useHostMemory));
    UNWRAP_OR_FWD_RESULT(copier, getCudaBufferCopierFactory()->createBufferCopier(commandQueue,
                                                                                 hipMemcpyDeviceToDevice));
    return createRelocatableResizableBufferFactory(allocator.get(), copier.get());
  }

  [[nodiscard]] virtual Result<IBufferFactory> createSysMemBufferFactory() noexcept {
    return createBufferFactory(getSysMemAllocator());
  }

  ABSTRACT_IREF(IFactories);
};

GS_EXPORT [[nodiscard]] Result<IFactories> getFactoriesSingleton() noexcept;

#endif  // GPUSDRPIPELINE_FACTORIES_H
