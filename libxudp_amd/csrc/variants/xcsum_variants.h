/* variants/xcsum_variants.h -- A/B kernels kept OUT of libxcsum.so.
 *
 * Both lost their measurements against the product kernels and
 * are built only into `make variant` libraries (libxudp_amd/variants/NAME/),
 * which link these objects next to the product's.  The product library
 * reaches them through the weak hooks declared in xcsum_internal.h
 * (variant_supported / launch_variant), which are null there.
 *   - csum_lds_kernel<K, D>: chunks moved by LDS-DMA into a D-deep ring,
 *     Geometry{16, 10 + D, K};
 *   - csum_seg_kernel<D, F, ATOM>: segmented stream for packed mixed sizes,
 *     Geometry{64, F, D}; Geometry{64, F, 100 + D}: the round-6 form whose
 *     finished spans go to LDS words by ds_add instead of a wave reduction. */
#ifndef XCSUM_VARIANTS_H
#define XCSUM_VARIANTS_H

#include "xcsum_internal.h"

/* (F frames per unit, D rows of 1 KiB in flight per wave) */
#define XCSUM_SEG_GEOMETRIES(X) X(64, 4) X(64, 8) X(16, 4)

namespace xcsum {
hipError_t launch_seg(const CsumArgs &a, int F, int D, int cus, int bpc, hipStream_t s);
}

#endif
