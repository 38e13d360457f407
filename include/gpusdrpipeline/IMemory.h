#pragma once
// Source-compatible include path of the reference; declarations live in gpusdrpipeline/abi/core.h.
#include <gpusdrpipeline/abi/core.h>
