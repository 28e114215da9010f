// fcg_status.hpp -- HIP status hygiene of the C ABI.  HIP keeps the status of the last failed
// runtime call until hipGetLastError() reads it, and the caller's next HIP call (torch's, in
// the Python host) would report it as its own failure ("invalid device ordinal" after a probe
// of a missing device).  Every entry point that returns FCG_ERR_DEVICE therefore reads it first.
#pragma once

#include <hip/hip_runtime.h>

#include "fourc_gpu.h"

// FCG_ERR_DEVICE with HIP's last error consumed
inline int fcg_device_error()
{
  (void)hipGetLastError();
  return FCG_ERR_DEVICE;
}

// hipSetDevice that leaves no sticky status behind when the device does not exist
inline bool fcg_use_device(int device)
{
  if (hipSetDevice(device) == hipSuccess) return true;
  (void)hipGetLastError();
  return false;
}
