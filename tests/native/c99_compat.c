/* The public header must compile as strict C99 (reference tests/c99_compat/enforce_c99_compat.c). */
#include "pccl.h"

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
