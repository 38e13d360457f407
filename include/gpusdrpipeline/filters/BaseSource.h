#pragma once
// Source-compatible include path of the reference; declarations live in gpusdrpipeline/abi/base_filters.h.
#include <gpusdrpipeline/abi/base_filters.h>
