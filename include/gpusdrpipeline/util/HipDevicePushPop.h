#pragma once
// Source-compatible include path of the reference; declarations live in gpusdrpipeline/abi/errors.h.
#include <gpusdrpipeline/abi/errors.h>
