/*
 * nxec_isal_compat.h -- source-level drop-in for the ISA-L erasure_code API
 * as the Nexoedge coding layer uses it.
 *
 * In /root/reference/src/common/coding/rs.cc:5-7 and coding_util.hh:4-6 replace
 *     extern "C" { #include <isa-l/erasure_code.h> }
 * with
 *     #include "nxec_isal_compat.h"
 * and link libnxec instead of libisal (src/common/CMakeLists.txt:5-8).  Every
 * ISA-L call on the path (rs.cc:26,27,89,104,106,196,219,229,230,290,316;
 * coding_util.hh:20,21,27,28) then resolves to the MI355X implementation with
 * identical arguments and layouts; ec_encode_data runs on the GPU.
 */
#ifndef NXEC_ISAL_COMPAT_H
#define NXEC_ISAL_COMPAT_H

#include "nxec.h"

#define ec_init_tables nxec_ec_init_tables      /* erasure_code.h:74  */
#define ec_encode_data nxec_ec_encode_data      /* erasure_code.h:98  */
#define gf_gen_rs_matrix nxec_gf_gen_rs_matrix  /* erasure_code.h:870 */
#define gf_mul nxec_gf_mul                      /* erasure_code.h:905 */
#define gf_invert_matrix nxec_gf_invert_matrix  /* erasure_code.h:931 */
#define gf_inv nxec_gf_inv

#endif
