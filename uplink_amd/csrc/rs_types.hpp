// Fixed-width integer types for the headers that are also compiled at run
// time by hiprtc (rs_encoder_registry.cpp), whose built-in runtime header
// keeps them in a namespace of its own.
#pragma once
#ifdef __HIPCC_RTC__
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::uint64_t uint64_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::int64_t int64_t;
#else
#include <stdint.h>
#endif
