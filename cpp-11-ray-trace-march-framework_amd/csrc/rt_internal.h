// rt_internal.h -- shared between the library's translation units (not part of the ABI).
#pragma once
#include <string>

// Sets the thread-local message rt_last_error returns; returns `code`.
int rt_internal_fail(int code, const std::string& msg);
// RT_OK when `device` is a visible gfx950 device (hipSetDevice done), else RT_E_NODEVICE/RT_E_HIP.
int rt_internal_use_device(int device, int *num_cus);
