/*
 * ccoip_inet.h — socket address POD types shared by the C API and the wire protocol.
 *
 * Layout-compatible with the reference's public header (ccoip/public_include/ccoip_inet.h)
 * so C programs written against pccl.h compile unchanged.
 */
#ifndef PCCL_AMD_CCOIP_INET_H
#define PCCL_AMD_CCOIP_INET_H

#ifdef __cplusplus
#include <cstdint>
extern "C" {
#else
#include <stdint.h>
#endif

typedef enum ccoip_inet_protocol_t {
    inetIPv4,
    inetIPv6
} ccoip_inet_protocol_t;

typedef struct ccoip_ipv4_address_t {
    uint8_t data[4];
} ccoip_ipv4_address_t;

typedef struct ccoip_ipv6_address_t {
    uint8_t data[16];
} ccoip_ipv6_address_t;

typedef struct ccoip_inet_address_t {
    ccoip_inet_protocol_t protocol;
    ccoip_ipv4_address_t ipv4;
    ccoip_ipv6_address_t ipv6;
} ccoip_inet_address_t;

typedef struct ccoip_socket_address_t {
    ccoip_inet_address_t inet;
    uint16_t port;
} ccoip_socket_address_t;

#ifdef __cplusplus
}
#endif

#endif /* PCCL_AMD_CCOIP_INET_H */
