/* The public header must compile as strict C99 (reference tests/c99_compat/enforce_c99_compat.c). */
#include "pccl.h"

/* ABI pin: the reference's pcclBuildInfo_t is exactly one bool (reference include/pccl.h:212-217); a caller built
 * against that header allocates sizeof == 1 and pcclGetBuildInfo must not write more. */
typedef char pccl_build_info_abi_check[(sizeof(pcclBuildInfo_t) == sizeof(bool)) ? 1 : -1];
typedef char pccl_reduce_info_abi_check[(sizeof(pcclReduceInfo_t) == 24) ? 1 : -1];
typedef char pccl_quant_opts_abi_check[(sizeof(pcclQuantizationOptions_t) == 8) ? 1 : -1];

int pccl_c99_probe(void) {
    pcclReduceDescriptor_t d;
    d.count = 1;
    d.op = pcclSum;
    d.tag = 0;
    d.src_descriptor.datatype = pcclFloat;
    d.src_descriptor.distribution_hint = pcclDistributionNone;
    d.quantization_options.quantized_datatype = pcclFloat;
    d.quantization_options.algorithm = pcclQuantNone;
    return (int) d.count + (int) sizeof(pcclCommCreateParams_t) * 0;
}
