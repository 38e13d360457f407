#pragma once
// Source-compatible include path of the reference; declarations live in gpusdrpipeline/abi/queue.h.
#include <gpusdrpipeline/abi/queue.h>
