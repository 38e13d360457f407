#pragma once
// Source-compatible include path of the reference; declarations live in gpusdrpipeline/abi/buffers.h.
#include <gpusdrpipeline/abi/buffers.h>
