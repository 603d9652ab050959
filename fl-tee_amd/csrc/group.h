// group.h — an enclave id spanning several GPUs (group.hip).
#pragma once
#include "common.h"
#include "engine.h"

namespace fltee {

struct Group;
// returned by the group paths when the shape is not sharded there (the caller runs
// the single-device path on the root)
constexpr uint32_t FLTEE_GROUP_FALLBACK = 0xFFFFFFFEu;

Group *group_create(const int *devs, int n, uint32_t *status);
void group_destroy(Group *G);
int group_size(const Group *G);
int group_root_device(const Group *G);
hipStream_t group_root_stream(const Group *G);

// dense uploads straight from the host ciphertext, parameter-range sharded; rk_host =
// the n clients' AES round keys (44 words each); d_out_root gets the averaged f32[d].
// A record out of position: reject_order (baseline / path_oram, fixed cost) -> 0x2, else
// FLTEE_GROUP_FALLBACK (non_oblivious reruns it with scatter semantics on the root)
uint32_t group_dense_ecall(Group *G, const uint32_t *rk_host, size_t n, const uint8_t *enc,
                           size_t d, float coef, float *d_out_root, float *t_load, float *t_dec,
                           bool reject_order);
// Where the client-major n x k records come from: decrypted into the root device's HBM
// (root_rec), or the host ciphertext (enc, bpc bytes per client, rk = the clients' round
// keys): then every GPU of the eid copies and decrypts the clients covering its own
// range (t_load / t_dec: the ECALL's "Loading" / "Decryption" times).
struct GroupInput {
    const uint64_t *root_rec = nullptr;
    const uint8_t *enc = nullptr;
    const uint32_t *rk = nullptr;
    size_t bpc = 0;
    float *t_load = nullptr, *t_dec = nullptr;
};
uint32_t group_advanced(Group *G, const GroupInput &in, size_t n, size_t k, size_t d, float coef,
                        float *d_out_root);
uint32_t group_nips19(Group *G, DeviceCtx *root, const GroupInput &in, size_t n, size_t k,
                      size_t k_req, size_t d, uint64_t seed, float coef, float *d_out_root);
// halo: the fold halo of every batch (n, or the exact-runs policy's worst case)
uint32_t group_optimized(Group *G, const GroupInput &in, size_t n, size_t k, size_t d,
                         size_t batch, float coef, float *d_out_root, size_t halo);
// true when the group loads the host ciphertext per GPU (eids of > 1 rank)
bool group_splits_host_copy(const Group *G);

}  // namespace fltee
