// Symbol visibility for the ldpc_ece535a blocks (reference:
// include/ldpc_ece535a/api.h of gr-ldpc_ece535a).
#ifndef INCLUDED_LDPC_ECE535A_API_H
#define INCLUDED_LDPC_ECE535A_API_H
#define LDPC_ECE535A_API __attribute__((visibility("default")))
#endif
