// SteppingDriver (reference src/driver/SteppingDriver.cpp:102-496); see driver.h for the
// differences from the reference.
#include "driver.h"

#include "buffers.h"
#include "graph_state.h"

#include <gpusdrpipeline/abi/errors.h>
#include <gsdr/gsdr_amd.h>

#include <algorithm>
#include <cstring>

namespace gsdr_rt {

namespace {
constexpr int kMaxDepth = 1024;  // longer upstream chains than this are treated as a cycle
const char kUnnamed[] = "NOT SET";  // SteppingDriver.cpp:30
}  // namespace

SteppingDriver::SourceInfo& SteppingDriver::sourceInfo(Source* source) {
  auto [it, inserted] = mSources.try_emplace(source, source);
  if (inserted) mSourceOrder.push_back(source);
  return it->second;
}

SteppingDriver::SinkInfo& SteppingDriver::sinkInfo(Sink* sink) { return mSinks.try_emplace(sink, sink).first->second; }

const char* SteppingDriver::nameOf(Node* node) const noexcept {
  auto it = mNodes.find(node);
  return it == mNodes.end() ? kUnnamed : it->second.name.c_str();
}

// SteppingDriver.cpp:102-135. A sink port takes one upstream; connecting a second is InvalidState.
Status SteppingDriver::connect(Source* source, size_t sourcePort, Sink* sink, size_t sinkPort) noexcept {
  if (source == nullptr || sink == nullptr) {
    gsloge("SteppingDriver::connect: source and sink must not be null");
    return Status_InvalidArgument;
  }
  try {
    auto existing = mSinks.find(sink);
    if (existing != mSinks.end() && sinkPort < existing->second.inputs.size() &&
        existing->second.inputs[sinkPort].source != nullptr) {
      const Upstream& up = existing->second.inputs[sinkPort];
      gsloge("Sink [%s] port [%zu] is already connected to Source [%s] port [%zu]", nameOf(sink), sinkPort,
             nameOf(up.source), up.port);
      return Status_InvalidState;
    }
    SourceInfo& si = sourceInfo(source);
    if (si.ports.size() <= sourcePort) si.ports.resize(sourcePort + 1);
    si.ports[sourcePort].push_back(SinkPortKey{sink, sinkPort});

    SinkInfo& ki = sinkInfo(sink);
    if (ki.inputs.size() <= sinkPort) ki.inputs.resize(sinkPort + 1);
    ki.inputs[sinkPort] = Upstream{source, sourcePort};
    mStepNodesValid = false;

    if (Sink* s = source->asSink()) mTails.erase(std::remove(mTails.begin(), mTails.end(), s), mTails.end());
    Source* sinkAsSource = sink->asSource();
    if ((sinkAsSource == nullptr || mSources.find(sinkAsSource) == mSources.end()) &&
        std::find(mTails.begin(), mTails.end(), sink) == mTails.end()) {
      mTails.push_back(sink);
    }
    return Status_Success;
  }
  IF_CATCH_RETURN_STATUS;
}

// SteppingDriver.cpp:137-141
Status SteppingDriver::setupNode(Node* node, const char* functionInGraph) noexcept {
  if (node == nullptr) return Status_InvalidArgument;
  try {
    auto [it, inserted] = mNodes.try_emplace(node, node, functionInGraph);
    if (inserted) mNodeOrder.push_back(node);
    else it->second.name = functionInGraph != nullptr ? functionInGraph : "";
    return Status_Success;
  }
  IF_CATCH_RETURN_STATUS;
}

void SteppingDriver::iterateOverConnections(void* context,
                                            void (*connectionIterator)(IDriver*, void*, Source*, size_t, Sink*,
                                                                       size_t) noexcept) noexcept {
  if (connectionIterator == nullptr) return;
  for (Source* source : mSourceOrder) {
    const SourceInfo& si = mSources.at(source);
    for (size_t p = 0; p < si.ports.size(); ++p)
      for (const SinkPortKey& k : si.ports[p]) connectionIterator(this, context, source, p, k.sink, k.port);
  }
}

void SteppingDriver::iterateOverNodes(void* context, void (*nodeIterator)(IDriver*, void*, Node*) noexcept) noexcept {
  if (nodeIterator == nullptr) return;
  for (Node* n : mNodeOrder) nodeIterator(this, context, n);
}

// The reference keeps no attributes (SteppingDriver.cpp:174-182).
void SteppingDriver::iterateOverNodeAttributes(Node*, void*,
                                               void (*)(IDriver*, Node*, void*, const char*, const char*) noexcept)
    noexcept {}

// SteppingDriver.cpp:465-496: this driver's names first, then nested drivers'.
size_t SteppingDriver::getNodeName(Node* node, char* name, size_t nameBufLen, bool* foundOut) noexcept {
  bool found = false;
  size_t len = 0;
  auto it = mNodes.find(node);
  if (it != mNodes.end()) {
    const std::string& s = it->second.name;
    len = s.size();
    if (name != nullptr && nameBufLen > 0) {
      const size_t n = std::min(len, nameBufLen);
      std::memcpy(name, s.data(), n);
      if (nameBufLen > len) name[len] = 0;
    }
    found = true;
  } else {
    for (Node* n : mNodeOrder) {
      IDriver* d = n->asDriver();
      if (d == nullptr || d == this) continue;
      len = d->getNodeName(node, name, nameBufLen, &found);
      if (found) break;
    }
    if (!found) {
      len = 0;
      if (name != nullptr && nameBufLen > 0) name[0] = 0;
    }
  }
  if (foundOut != nullptr) *foundOut = found;
  return len;
}

// SteppingDriver.cpp:453-463: every connected output port has bytes to give.
bool SteppingDriver::hasDataForAllPorts(Source* source) {
  auto it = mSources.find(source);
  if (it == mSources.end()) return true;
  for (size_t p = 0; p < it->second.ports.size(); ++p)
    if (source->getOutputDataSize(p) == 0) return false;
  return true;
}

// SteppingDriver.cpp:193-199
Status SteppingDriver::doFilter() noexcept {
  try {
    for (size_t i = 0; i < mTails.size(); ++i) FWD_IF_ERR(doSinkInput(mTails[i], 0));
    return Status_Success;
  }
  IF_CATCH_RETURN_STATUS;
}

// SteppingDriver.cpp:201-245: pull every upstream of `sink` (recursing through filters that have
// no output yet), then move one chunk from each upstream into it. A filter that still has nothing
// after being fed ends this sink's step.
Status SteppingDriver::doSinkInput(Sink* sink, int depth) {
  auto it = mSinks.find(sink);
  if (it == mSinks.end()) return Status_Success;  // fed from outside this driver
  if (depth > kMaxDepth) {
    gsloge("SteppingDriver: upstream chain of [%s] is longer than %d nodes (cycle?)", nameOf(sink), kMaxDepth);
    return Status_InvalidState;
  }
  const size_t nInputs = it->second.inputs.size();
  for (size_t port = 0; port < nInputs; ++port) {
    const Upstream up = it->second.inputs[port];
    if (up.source == nullptr) {
      gslogt("Sink [%s] port [%zu] does not have a Source connected to it", nameOf(sink), port);
      continue;
    }
    if (Fir* fir = fusableFirAm(up.source)) {  // Fir -> QuadAmDemod in one launch
      if (fir->fusedAmOutputBytes() == 0) {
        FWD_IF_ERR(doSinkInput(fir, depth + 1));
        if (fir->fusedAmOutputBytes() == 0) return Status_Success;
      }
      FWD_IF_ERR(doSourceOutput(up.source, fir));
      ++mStats.fused;
      continue;
    }
    Sink* upstreamSink = up.source->asSink();
    if (upstreamSink != nullptr && !hasDataForAllPorts(up.source)) {
      FWD_IF_ERR(doSinkInput(upstreamSink, depth + 1));
      if (!hasDataForAllPorts(up.source)) return Status_Success;
    }
    if (hasDataForAllPorts(up.source)) FWD_IF_ERR(doSourceOutput(up.source));
  }
  return Status_Success;
}

// The Fir feeding `source` when `source` is a QuadAmDemod the driver may step together with it: the
// AM window is empty (nothing of an unfused step left to demodulate), its one input is fed by a
// Fir with real taps whose only sink it is, both on one stream.
Fir* SteppingDriver::fusableFirAm(Source* source) {
  if (!mFuseFirAm) return nullptr;
  auto* am = dynamic_cast<QuadAmDemod*>(source);
  if (am == nullptr || !am->inputEmpty() || mSources.find(source) == mSources.end()) return nullptr;
  auto it = mSinks.find(am);
  if (it == mSinks.end() || it->second.inputs.size() != 1 || it->second.inputs[0].port != 0) return nullptr;
  auto* fir = dynamic_cast<Fir*>(it->second.inputs[0].source);
  if (fir == nullptr || !fir->canFuseAm() || fir->stream() != am->stream()) return nullptr;
  auto fs = mSources.find(fir);
  if (fs == mSources.end() || fs->second.ports.size() != 1 || fs->second.ports[0].size() != 1) return nullptr;
  return fir;
}

// SteppingDriver.cpp:247-366: each connected sink lends a buffer sized
// alignUp(min(sink preferred, source available), source alignment); the first sink of a port
// receives readOutput's data, further sinks of the same port get a copy through the source's
// output copier; then every sink commits the bytes written. With `fusedFir` (source is the
// QuadAmDemod it feeds, fusableFirAm) the data comes from the fused FIR + AM launch instead.
Status SteppingDriver::doSourceOutput(Source* source, Fir* fusedFir) {
  SourceInfo& si = mSources.at(source);
  const size_t nPorts = si.ports.size();
  for (size_t p = 0; p < nPorts; ++p) {
    if (si.ports[p].empty()) {
      gsloge("Source [%s] must have a sink connected to port [%zu]", nameOf(source), p);
      return Status_InvalidState;
    }
  }
  mBufferRefs.clear();
  mPortBuffers.assign(nPorts, nullptr);
  // sinks that lent a buffer, so a failure can cancel their checkout (commit of 0 bytes)
  auto cancel = [&](size_t lentCount) {
    size_t i = 0;
    for (size_t p = 0; p < nPorts && i < lentCount; ++p)
      for (const SinkPortKey& k : si.ports[p]) {
        if (i++ >= lentCount) break;
        (void)k.sink->commitBuffer(k.port, 0);
      }
  };
  for (size_t p = 0; p < nPorts; ++p) {
    size_t alignment = source->getOutputSizeAlignment(p);
    if (alignment == 0) alignment = 1;
    const size_t available = fusedFir != nullptr ? fusedFir->fusedAmOutputBytes() : source->getOutputDataSize(p);
    for (const SinkPortKey& k : si.ports[p]) {
      const size_t want = std::min(k.sink->preferredInputBufferSize(k.port), available);
      const size_t bytes = want > SIZE_MAX - alignment + 1 ? want / alignment * alignment
                                                           : (want + alignment - 1) / alignment * alignment;
      Result<IBuffer> r = k.sink->requestBuffer(k.port, bytes);
      if (r.status != Status_Success) {
        gsloge("Sink [%s] port [%zu] could not lend %zu bytes", nameOf(k.sink), k.port, bytes);
        cancel(mBufferRefs.size());
        return r.status;
      }
      mBufferRefs.emplace_back(r.value);
      if (mPortBuffers[p] == nullptr) mPortBuffers[p] = r.value;
    }
  }
  // Fan-out: readOutput fills the port's first buffer and the driver copies it into the other
  // sinks' buffers, so the first buffer is capped (a view of the same memory) to the least room
  // any sink of the port lent; a sink that lent more simply receives fewer bytes this step.
  for (size_t p = 0; p < nPorts; ++p) {
    if (si.ports[p].size() < 2) continue;
    size_t firstRef = 0;
    for (size_t q = 0; q < p; ++q) firstRef += si.ports[q].size();
    size_t room = SIZE_MAX;
    for (size_t s = 0; s < si.ports[p].size(); ++s)
      room = std::min(room, mBufferRefs[firstRef + s]->range()->remaining());
    IBuffer* first = mBufferRefs[firstRef].get();
    if (first->range()->remaining() > room) {
      Ref<IBufferRangeMutableCapacity> range = new (std::nothrow) BufferRange();
      Ref<IBuffer> view = range.get() ? new (std::nothrow) BufferSlice(first, 0, range.get()) : nullptr;
      Status vs = view.get() ? Status_Success : Status_OutOfMemory;
      if (vs == Status_Success) {
        range->setCapacity(first->range()->endOffset() + room);
        vs = range->setUsedRange(first->range()->offset(), first->range()->endOffset());
      }
      if (vs != Status_Success) {
        cancel(mBufferRefs.size());
        return vs;
      }
      mPortBuffers[p] = view.get();
      mViewRefs.emplace_back(std::move(view));
    }
  }
  Status st = fusedFir != nullptr ? fusedFir->readOutputAm(mPortBuffers[0]) : source->readOutput(mPortBuffers.data(), nPorts);
  if (st != Status_Success) {
    gsloge("Source [%s] readOutput failed [%u]", nameOf(source), (unsigned)st);
    cancel(mBufferRefs.size());
    mViewRefs.clear();
    return st;
  }
  // copy to the other sinks of each port; on any failure every checkout is cancelled (committing
  // 0 bytes), so no sink stays checked out
  size_t ref = 0;
  std::vector<size_t> portBytes(nPorts, 0);
  for (size_t p = 0; p < nPorts; ++p) {
    IBuffer* populated = mPortBuffers[p];
    const size_t bytes = populated->range()->used();
    portBytes[p] = bytes;
    ++ref;  // the populated buffer
    for (size_t s = 1; s < si.ports[p].size(); ++s, ++ref) {
      IBuffer* target = mBufferRefs[ref].get();
      IBufferCopier* copier = source->getOutputCopier(p);
      Status cs = Status_Success;
      if (copier == nullptr) {
        gsloge("Source [%s] port [%zu] feeds %zu sinks but has no output copier", nameOf(source), p,
               si.ports[p].size());
        cs = Status_InvalidState;
      } else if (target->range()->remaining() < bytes) {
        cs = Status_OutOfRange;  // unreachable: the first buffer was capped to the least room
      } else {
        cs = copier->copy(target->writePtr(), populated->readPtr(), bytes);
        if (cs == Status_Success) cs = target->range()->increaseEndOffset(bytes);
      }
      if (cs != Status_Success) {
        cancel(mBufferRefs.size());
        mViewRefs.clear();
        return cs;
      }
    }
  }
  mViewRefs.clear();
  Status firstErr = Status_Success;
  for (size_t p = 0; p < nPorts; ++p)
    for (const SinkPortKey& k : si.ports[p]) {
      // every sink commits (or cancels) even after an earlier commit failed
      const Status cs = k.sink->commitBuffer(k.port, firstErr == Status_Success ? portBytes[p] : 0);
      if (firstErr == Status_Success && cs != Status_Success) firstErr = cs;
    }
  if (firstErr != Status_Success) {
    mBufferRefs.clear();
    return firstErr;
  }
  mBufferRefs.clear();
  return Status_Success;
}

// ---- graph stepping -----------------------------------------------------------------------------
// The steady state of a chain fed fixed-size chunks repeats: every node's window sits at one of a
// few placements (lazy compaction cycles through them), and a step from a given placement enqueues
// the same launches with the same arguments and leaves the same host state behind. So the step is
// captured once per placement - its device work as a hipGraph, its host outcome as every node's
// window state (which allocation is live, used range, checkout flags) - and a replay reinstates
// that host state and launches the graph: no per-node host logic, no per-kernel launches. A
// placement is captured only the second time it is seen (the first time may still grow windows:
// allocation, no replay), and the driver falls back to plain steps for good when a chain's state
// does not repeat (a tone source's phase) or a node is not on `stream`.

SteppingDriver::~SteppingDriver() {
  for (const CachedGraph& g : mGraphs) {
    (void)hipGraphExecDestroy(g.exec);
    (void)hipGraphDestroy(g.graph);
  }
}

namespace {

// The kernel launches of a captured step, in order, when its graph is a linear chain of kernel
// nodes (each node at most one dependency and one dependent); empty otherwise (memcpy / memset nodes,
// forks): such graphs replay through hipGraphLaunch.
std::vector<hipKernelNodeParams> linearKernelChain(hipGraph_t graph) {
  std::vector<hipKernelNodeParams> out;
  size_t n = 0;
  if (hipGraphGetNodes(graph, nullptr, &n) != hipSuccess || n == 0 || n > 8) return out;
  std::vector<hipGraphNode_t> nodes(n);
  if (hipGraphGetNodes(graph, nodes.data(), &n) != hipSuccess) return out;
  hipGraphNode_t cur = nullptr;
  for (hipGraphNode_t v : nodes) {
    hipGraphNodeType t;
    size_t deps = 0, dependents = 0;
    if (hipGraphNodeGetType(v, &t) != hipSuccess || t != hipGraphNodeTypeKernel ||
        hipGraphNodeGetDependencies(v, nullptr, &deps) != hipSuccess ||
        hipGraphNodeGetDependentNodes(v, nullptr, &dependents) != hipSuccess || deps > 1 || dependents > 1)
      return {};
    if (deps == 0) {
      if (cur != nullptr) return {};  // two roots: not a chain
      cur = v;
    }
  }
  while (cur != nullptr) {
    hipKernelNodeParams p{};
    if (hipGraphKernelNodeGetParams(cur, &p) != hipSuccess || p.func == nullptr || p.extra != nullptr) return {};
    out.push_back(p);
    size_t k = 1;
    hipGraphNode_t next = nullptr;
    if (hipGraphNodeGetDependentNodes(cur, &next, &k) != hipSuccess) return {};
    cur = k == 1 ? next : nullptr;
  }
  if (out.size() != n) out.clear();
  return out;
}

}  // namespace

bool SteppingDriver::chainState(hipStream_t stream, uint64_t& key) noexcept {
  if (!mStepNodesValid) {  // every connected node, in a fixed order (by address)
    mStepNodes.clear();
    mStepNodesOk = false;
    mStepNodesValid = true;
    try {
      std::vector<Node*> nodes;
      for (Source* so : mSourceOrder) nodes.push_back(so);
      for (const auto& kv : mSinks) nodes.push_back(kv.first);
      std::sort(nodes.begin(), nodes.end());
      nodes.erase(std::unique(nodes.begin(), nodes.end()), nodes.end());
      for (Node* n : nodes) {
        auto* g = dynamic_cast<IGraphStepState*>(n);
        if (g == nullptr) return false;
        mStepNodes.push_back(g);
      }
    } catch (...) {
      mStepNodes.clear();
      return false;
    }
    mStepNodesOk = !mStepNodes.empty();
  }
  if (!mStepNodesOk) return false;
  // process-wide kernel settings that become captured launch arguments: a replay must not run with
  // values that changed since its capture (kernel policy, FFT guard ratio, WS spin limit)
  const float guard = gsdrAmdGetFftGuard();
  uint32_t guardBits = 0;
  std::memcpy(&guardBits, &guard, sizeof guardBits);
  uint64_t h = 0xCBF29CE484222325ull ^ (uint64_t)gsdrAmdGetKernelPolicy();
  h = (h ^ guardBits) * 0x100000001B3ull;
  h = (h ^ (uint32_t)gsdrAmdGetWsSpinLimit()) * 0x100000001B3ull;
  h = (h ^ (mFuseFirAm ? 0x2u : 0x1u)) * 0x100000001B3ull;  // fused and unfused steps capture different work
  for (IGraphStepState* g : mStepNodes) {
    if (g->graphStream() != stream || !g->graphState(h)) return false;
    h = (h ^ reinterpret_cast<uintptr_t>(g)) * 0x100000001B3ull;
  }
  key = h;
  return true;
}

Status SteppingDriver::captureStep(hipStream_t stream, hipGraph_t* graphOut) noexcept {
  *graphOut = nullptr;
  SAFE_HIP_OR_RET_STATUS(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
  const Status st = doFilter();
  const hipError_t e = hipStreamEndCapture(stream, graphOut);
  if (st != Status_Success) {
    if (*graphOut != nullptr) (void)hipGraphDestroy(*graphOut);
    *graphOut = nullptr;
    return st;
  }
  SAFE_HIP_OR_RET_STATUS(e);
  return Status_Success;
}

Status SteppingDriver::doFilterGraphed(hipStream_t stream) noexcept {
  try {
    // a wave-specialised kernel inside an earlier replay that gave up a hand-off wait (the eager
    // entry points never see graph launches): a host peek; when set, settle and report it
    if (!mGraphs.empty()) {
      int dev = 0;
      if (hipStreamGetDevice(stream, &dev) == hipSuccess && gsdrAmdWsAbortsPending(dev) != 0) {
        SAFE_HIP_OR_RET_STATUS(hipStreamSynchronize(stream));
        if (gsdrAmdWsTakeAborts(dev) != 0) {
          gsloge("SteppingDriver: a wave-specialised kernel in a replayed step aborted (hand-off wait timed out)");
          return Status_RuntimeError;
        }
      }
    }
    uint64_t key = 0;
    if (mGraphOff || stream == nullptr || !chainState(stream, key)) {
      ++mStats.eager;
      return doFilter();
    }
    for (const CachedGraph& g : mGraphs) {
      if (g.key != key) continue;
      for (const auto& [node, state] : g.post) FWD_IF_ERR(node->restoreStepState(state));
      if (g.kernels.empty()) {
        SAFE_HIP_OR_RET_STATUS(hipGraphLaunch(g.exec, stream));
      } else {
        for (const hipKernelNodeParams& k : g.kernels)
          SAFE_HIP_OR_RET_STATUS(hipLaunchKernel(k.func, k.gridDim, k.blockDim, k.kernelParams, k.sharedMemBytes, stream));
        ++mStats.direct;
      }
      ++mStats.replayed;
      mGraphMisses = 0;
      return Status_Success;
    }
    if (std::find(mSeen.begin(), mSeen.end(), key) == mSeen.end()) {
      if (mSeen.size() >= 64 || ++mGraphMisses > 32) {
        mGraphOff = true;  // the state does not repeat: plain steps from now on
      } else {
        mSeen.push_back(key);
      }
      ++mStats.eager;
      return doFilter();
    }
    if (mGraphs.size() >= 16) {  // more placements than a steady state cycles through
      mGraphOff = true;
      ++mStats.eager;
      return doFilter();
    }
    hipGraph_t graph = nullptr;
    FWD_IF_ERR(captureStep(stream, &graph));
    if (graph == nullptr) return Status_RuntimeError;
    hipGraphExec_t exec = nullptr;
    const hipError_t ie = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    if (ie != hipSuccess) (void)hipGraphDestroy(graph);
    SAFE_HIP_OR_RET_STATUS(ie);
    CachedGraph cg{key, exec, graph, linearKernelChain(graph), {}};
    bool saved = true;
    cg.post.reserve(mStepNodes.size());
    for (IGraphStepState* n : mStepNodes) {
      cg.post.emplace_back(n, GraphNodeState{});
      saved = saved && n->saveStepState(cg.post.back().second);
    }
    const hipError_t le = hipGraphLaunch(exec, stream);
    const Status ls = le == hipSuccess ? Status_Success : Status_RuntimeError;
    if (saved && ls == Status_Success) {
      mGraphs.push_back(std::move(cg));
    } else {
      if (ls == Status_Success) SAFE_HIP_OR_RET_STATUS(hipStreamSynchronize(stream));
      (void)hipGraphExecDestroy(exec);
      (void)hipGraphDestroy(graph);
    }
    FWD_IF_ERR(ls);
    ++mStats.captured;
    return Status_Success;
  }
  IF_CATCH_RETURN_STATUS;
}

}  // namespace gsdr_rt
