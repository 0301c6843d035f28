/*
 * ccoip.h — CCoIP protocol constants (well-known ports).
 *
 * Port numbers follow the reference (ccoip/public_include/ccoip.h:11-29). Note the reference's pccl.h comments
 * disagree with this header about which of 48149/48150 is P2P vs shared state; we follow the
 * values that the Python API of the reference actually uses: p2p 48149, shared state 48150, benchmark 48151.
 * Every listener "bumps" to the next free port if the requested one is taken, so these are only defaults.
 */
#ifndef PCCL_AMD_CCOIP_H
#define PCCL_AMD_CCOIP_H

#define CCOIP_PROTOCOL_PORT_MASTER 48148
#define CCOIP_PROTOCOL_PORT_P2P 48149
#define CCOIP_PROTOCOL_PORT_SHARED_STATE 48150
#define CCOIP_PROTOCOL_PORT_BANDWIDTH_BENCHMARK 48151

#endif /* PCCL_AMD_CCOIP_H */
