// tdt_enc_ws.hip — the encode kernels of ONE word size (PSY_INST_WS), explicitly
// instantiated; psyne_amd/build.py compiles this file once per supported word size, in
// parallel with tdt_api.hip (which declares the same instances extern and launches them).
#define PSY_ENC_INST_TU 1
#include <hip/hip_runtime.h>

#include "tdt_encode.h"

#ifndef PSY_INST_WS
#error "PSY_INST_WS (the word size) must be defined"
#endif

#define PSY_ENC_DEF(WS, T, G, M, L, TL, PS, PA) \
    template __global__ void psy::tdt_encode_kernel<WS, T, G, psy::M, L, TL, PS, PA>(psy::EncodeArgs);
PSY_ENC_INSTANCES(PSY_ENC_DEF, PSY_INST_WS)
template __global__ void psy::tdt_encode_lscan_kernel<PSY_INST_WS>(psy::EncodeArgs, const uint32_t *, uint32_t);
