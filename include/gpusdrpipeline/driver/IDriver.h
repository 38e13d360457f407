#pragma once
// Source-compatible include path of the reference; declarations live in gpusdrpipeline/abi/graph.h.
#include <gpusdrpipeline/abi/graph.h>
