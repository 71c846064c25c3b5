/* Scalar typedefs used by the zfp API (reference: include/zfp/internal/zfp/types.h:4-123). */
#ifndef ZFP_TYPES_H
#define ZFP_TYPES_H

#include <stdint.h>

typedef unsigned char uchar;
typedef unsigned short ushort;
typedef unsigned int uint;
typedef unsigned long ulong;

typedef int8_t int8;
typedef uint8_t uint8;
typedef int16_t int16;
typedef uint16_t uint16;
typedef int32_t int32;
typedef uint32_t uint32;
typedef int64_t int64;
typedef uint64_t uint64;

#ifndef UINT64C
#define UINT64C(x) ((uint64)(x##ull))
#endif

#endif
