// SteppingDriver: the pull-based caller of the filter graph (reference src/driver/SteppingDriver.cpp,
// semantics of :102-141 connect/setupNode and :193-366 doFilter/doSinkInput/doSourceOutput).
//
// Host-side bookkeeping only; every readOutput() it makes enqueues on the node's own HIP stream.
// Differences from the reference, all deliberate:
//  * a sink port records its upstream once (the reference inserts it twice, :121-124);
//  * graph tails are stepped in connection order (an unordered_set in the reference), so a step is
//    reproducible;
//  * node names are looked up only when a message is logged (the reference builds std::string
//    names on every step, :208-217);
//  * a cycle in the graph ends the step with Status_InvalidState instead of recursing forever.
//
// MI355X extension: doFilterGraphed(stream) - the same step, with its device work replayed from a
// captured hipGraph once the chain's host state repeats, and its host work replaced by reinstating
// the host state the captured step left behind (see driver.cpp).
#pragma once

#include <gpusdrpipeline/Factories.h>

#include "filters.h"
#include "graph_state.h"

#include <hip/hip_runtime_api.h>

#include <string>
#include <unordered_map>
#include <vector>

namespace gsdr_rt {

class SteppingDriver final : public ISteppingDriver {
 public:
  SteppingDriver() noexcept = default;

  Status connect(Source* source, size_t sourcePort, Sink* sink, size_t sinkPort) noexcept final;
  Status setupNode(Node* node, const char* functionInGraph) noexcept final;
  void iterateOverConnections(void* context,
                              void (*connectionIterator)(IDriver* driver, void* context, Source* source,
                                                         size_t sourcePort, Sink* sink,
                                                         size_t sinkPort) noexcept) noexcept final;
  void iterateOverNodes(void* context,
                        void (*nodeIterator)(IDriver* driver, void* context, Node* node) noexcept) noexcept final;
  void iterateOverNodeAttributes(Node* node, void* context,
                                 void (*nodeAttrIterator)(IDriver* driver, Node* node, void* context,
                                                          const char* attrName,
                                                          const char* attrVal) noexcept) noexcept final;
  size_t getNodeName(Node* node, char* name, size_t nameBufLen, bool* foundOut) noexcept final;
  Status doFilter() noexcept final;

  // One doFilter() step; when every node is a graph-steppable filter on `stream` and the chain's
  // host state (window placement of every node) has been seen before, the step's device work is
  // captured once into a hipGraph keyed by that state and replayed from then on.
  Status doFilterGraphed(hipStream_t stream) noexcept;
  struct GraphStats {
    size_t eager = 0;     // steps run as plain launches
    size_t captured = 0;  // steps that captured (and launched) a new graph
    size_t replayed = 0;  // steps whose device work was a cached graph launch
    size_t direct = 0;    // of those: replayed as direct kernel launches (a linear chain of kernel nodes)
    size_t fused = 0;     // Fir -> QuadAmDemod edges moved as one fused launch
  };
  GraphStats graphStats() const noexcept { return mStats; }

  // MI355X: a Fir (real taps, cf32 or int8 IQ input) whose only sink is a QuadAmDemod on the same
  // stream is stepped together with it - ONE gsdrFirFCAmDemod launch writes |y| straight into the
  // QuadAmDemod's downstream buffer, so the cf32 FIR output never goes through HBM and the AM node's
  // launch disappears (bit-identical output; the AM node's window stays empty). On by default.
  // Part of the cached graphs' key (chainState): toggling it never replays a step captured in the
  // other mode.
  void setFuseFirAm(bool on) noexcept { mFuseFirAm = on; }

 private:
  struct SinkPortKey {
    Sink* sink;
    size_t port;
  };
  struct Upstream {  // what feeds one sink port
    Source* source = nullptr;
    size_t port = 0;
  };
  struct SourceInfo {
    ImmutableRef<Source> source;
    std::vector<std::vector<SinkPortKey>> ports;  // source port -> connected sink ports, in connect order
    explicit SourceInfo(Source* s) : source(s) {}
  };
  struct SinkInfo {
    ImmutableRef<Sink> sink;
    std::vector<Upstream> inputs;  // sink port -> upstream (source == nullptr: unconnected)
    explicit SinkInfo(Sink* s) : sink(s) {}
  };
  struct NodeInfo {
    ImmutableRef<Node> node;
    std::string name;
    NodeInfo(Node* n, const char* nm) : node(n), name(nm != nullptr ? nm : "") {}
  };

  SourceInfo& sourceInfo(Source* source);
  SinkInfo& sinkInfo(Sink* sink);
  const char* nameOf(Node* node) const noexcept;
  bool hasDataForAllPorts(Source* source);
  Status doSinkInput(Sink* sink, int depth);
  Status doSourceOutput(Source* source, Fir* fusedFir = nullptr);
  Fir* fusableFirAm(Source* source);

  // std::unordered_map keeps element addresses stable across inserts (references handed out above)
  std::unordered_map<Source*, SourceInfo> mSources;
  std::unordered_map<Sink*, SinkInfo> mSinks;
  std::vector<Source*> mSourceOrder;  // first-connect order, for iterateOverConnections
  std::vector<Sink*> mTails;          // sinks whose node is not (yet) a connected source
  std::unordered_map<Node*, NodeInfo> mNodes;
  std::vector<Node*> mNodeOrder;
  // per-step scratch, kept to avoid reallocation on every doSourceOutput
  std::vector<Ref<IBuffer>> mBufferRefs;
  std::vector<IBuffer*> mPortBuffers;
  std::vector<Ref<IBuffer>> mViewRefs;  // capped fan-out views (doSourceOutput)
  // graph stepping
  struct CachedGraph {
    uint64_t key;
    hipGraphExec_t exec;
    hipGraph_t graph;  // kept: `kernels` point into its nodes' parameters
    // a step that captured as a linear chain of kernel nodes (the steady-state fused Fir -> AM step is
    // one) is replayed by launching those kernels with their captured parameters: hipGraphLaunch costs
    // more host time than the one or two launches it replaces
    std::vector<hipKernelNodeParams> kernels;
    // every node's host state after the captured step, reinstated on replay instead of running
    // the step's host logic again
    std::vector<std::pair<IGraphStepState*, GraphNodeState>> post;
  };
  std::vector<CachedGraph> mGraphs;
  std::vector<uint64_t> mSeen;
  size_t mGraphMisses = 0;
  bool mGraphOff = false;
  GraphStats mStats;
  // graph-steppable nodes in a fixed order (by address), rebuilt when a connection changes
  std::vector<IGraphStepState*> mStepNodes;
  bool mStepNodesValid = false;
  bool mStepNodesOk = false;
  bool mFuseFirAm = true;
  bool chainState(hipStream_t stream, uint64_t& key) noexcept;
  Status captureStep(hipStream_t stream, hipGraph_t* graphOut) noexcept;

  ~SteppingDriver() final;
  REF_COUNTED_NO_DESTRUCTOR(SteppingDriver);
};

class SteppingDriverFactory final : public ISteppingDriverFactory {
 public:
  Result<ISteppingDriver> createSteppingDriver() noexcept final {
    return makeRefResultNonNull<ISteppingDriver>(new (std::nothrow) SteppingDriver());
  }
  REF_COUNTED(SteppingDriverFactory);
};

}  // namespace gsdr_rt
