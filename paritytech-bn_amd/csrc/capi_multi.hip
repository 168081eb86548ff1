// capi_multi.hip -- the multi-device context of the C ABI:
// one process drives several MI355X of the node.
//
// Host-buffer calls shard their n elements contiguously over the devices --
// device k takes [k*n/D, (k+1)*n/D) -- run the shards concurrently (one host
// thread per device, each on its own single-device sub-context) and write each
// shard straight into the caller's output, so no exchange is needed.  The
// product forms (pairing_batch, miller_loop_batch; lib.rs:615-633) reduce each
// shard to one Miller value on its device; the D partials are multiplied on
// device 0 in device order and pairing_batch runs one final exponentiation --
// the same exact Fq12 product as the reference's single shared loop
// (mod.rs:609-640: squaring is a ring homomorphism and Fq12 is commutative).
//
// bn_pairing_many_allgather_dev is BASELINE config 4 in one process: each
// device computes its HBM-resident shard and one RCCL all-gather over xGMI
// leaves every device holding all results in device order.  RCCL is opened
// with dlopen on first use, so single-device users never load it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "ctx.h"

namespace {

int mfail(bn_ctx* c, int code, const std::string& msg) {
    if (c) {
        std::lock_guard<std::mutex> g(c->err_mu);
        c->err = msg;
    }
    return code;
}
// restores the calling thread's current device on scope exit
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

// contiguous shard k of n over d parts (the same split as substrate_bn/parallel.py)
void shard(size_t n, size_t d, size_t k, size_t* lo, size_t* hi) {
    *lo = n * k / d;
    *hi = n * (k + 1) / d;
}

// run fn(k, lo, hi) for every device shard concurrently; first error wins
template <class F>
int for_shards(bn_ctx* c, size_t n, F&& fn) {
    const size_t d = c->subs.size();
    std::vector<int> rc(d, BN_OK);
    std::vector<std::thread> th;
    for (size_t k = 0; k < d; ++k) {
        size_t lo, hi;
        shard(n, d, k, &lo, &hi);
        th.emplace_back([&, k, lo, hi] { rc[k] = hi > lo ? fn(k, lo, hi) : BN_OK; });
    }
    for (auto& t : th) t.join();
    for (size_t k = 0; k < d; ++k)
        if (rc[k] != BN_OK)
            return mfail(c, rc[k], "device " + std::to_string(c->devices[k]) + ": " + bn_last_error(c->subs[k]));
    return BN_OK;
}

// ---------------------------------------------------------------- RCCL through dlopen
// the few entry points used, typed after rccl.h (ncclResult_t = int, ncclUint8 = 1)
struct Rccl {
    void* so = nullptr;
    int (*comm_init_all)(void** comms, int ndev, const int* devlist) = nullptr;
    int (*all_gather)(const void* send, void* recv, size_t count, int dtype, void* comm, hipStream_t s) = nullptr;
    int (*group_start)() = nullptr;
    int (*group_end)() = nullptr;
    int (*comm_destroy)(void* comm) = nullptr;
    const char* (*error_string)(int) = nullptr;
};
constexpr int kNcclUint8 = 1;

int rccl_load(bn_ctx* c, Rccl* r) {
    r->so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!r->so) r->so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!r->so) return mfail(c, BN_ERR_HIP, std::string("dlopen librccl.so.1: ") + dlerror());
    r->comm_init_all = (int (*)(void**, int, const int*))dlsym(r->so, "ncclCommInitAll");
    r->all_gather = (int (*)(const void*, void*, size_t, int, void*, hipStream_t))dlsym(r->so, "ncclAllGather");
    r->group_start = (int (*)())dlsym(r->so, "ncclGroupStart");
    r->group_end = (int (*)())dlsym(r->so, "ncclGroupEnd");
    r->comm_destroy = (int (*)(void*))dlsym(r->so, "ncclCommDestroy");
    r->error_string = (const char* (*)(int))dlsym(r->so, "ncclGetErrorString");
    if (!r->comm_init_all || !r->all_gather || !r->group_start || !r->group_end || !r->comm_destroy ||
        !r->error_string)
        return mfail(c, BN_ERR_HIP, "librccl.so.1 lacks an expected symbol");
    return BN_OK;
}

struct Comms {
    Rccl r;
    std::vector<void*> comm;
};

int comms_get(bn_ctx* c, Comms** out) {
    if (!c->comms) {
        Comms* cm = new Comms();
        int rc = rccl_load(c, &cm->r);
        if (rc) {
            delete cm;
            return rc;
        }
        cm->comm.assign(c->devices.size(), nullptr);
        const int e = cm->r.comm_init_all(cm->comm.data(), (int)c->devices.size(), c->devices.data());
        if (e != 0) {
            std::string m = std::string("ncclCommInitAll: ") + cm->r.error_string(e);
            delete cm;
            return mfail(c, BN_ERR_HIP, m);
        }
        c->comms = cm;
    }
    *out = (Comms*)c->comms;
    return BN_OK;
}

}  // namespace

extern "C" {

void bn_shard_range(size_t n, int ndev, int k, size_t* lo, size_t* hi) {
    if (ndev <= 0 || k < 0 || k >= ndev || !lo || !hi) {
        if (lo) *lo = 0;
        if (hi) *hi = 0;
        return;
    }
    shard(n, (size_t)ndev, (size_t)k, lo, hi);
}

int bn_ctx_create_multi(const int* devices, int ndev, bn_ctx** out) {
    if (!out || !devices || ndev <= 0) return BN_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    bn_ctx* c = new bn_ctx();
    c->device = -1;
    for (int k = 0; k < ndev; ++k) {
        bn_ctx* s = nullptr;
        const int rc = bn_ctx_create(devices[k], &s);
        if (rc != BN_OK) {
            for (bn_ctx* d : c->subs) bn_ctx_destroy(d);
            c->subs.clear();
            delete c;
            return rc;
        }
        c->subs.push_back(s);
        c->devices.push_back(devices[k]);
    }
    *out = c;
    return BN_OK;
}

int bn_ctx_num_devices(const bn_ctx* c) {
    if (!c) return 0;
    return c->subs.empty() ? 1 : (int)c->subs.size();
}

bn_ctx* bn_ctx_device(bn_ctx* c, int k) {
    if (!c) return nullptr;
    if (c->subs.empty()) return k == 0 ? c : nullptr;
    return k >= 0 && k < (int)c->subs.size() ? c->subs[k] : nullptr;
}

int bn_pairing_many_allgather_dev(bn_ctx* c, const bn_g1* const* d_p, const bn_g2* const* d_q, size_t n_per_dev,
                                  bn_gt* const* d_out, void* const* streams) {
    if (!c || !d_p || !d_q || !d_out) return BN_ERR_INVALID_ARGUMENT;
    // a single-device context is a world of one (no collective)
    if (c->subs.empty()) return bn_pairing_many_dev(c, d_p[0], d_q[0], n_per_dev, d_out[0], streams ? streams[0] : nullptr);
    const std::vector<bn_ctx*>& subs = c->subs;
    const size_t d = subs.size();
    if (n_per_dev == 0) return BN_OK;
    std::lock_guard<std::mutex> lock(c->mu);  // the multi context's own lock: one collective at a time
    DeviceGuard keep_device;                  // the sub-context calls and the gather switch devices
    std::vector<hipStream_t> st(d);
    for (size_t k = 0; k < d; ++k) {
        st[k] = streams && streams[k] ? (hipStream_t)streams[k] : (hipStream_t)bn_ctx_stream(subs[k]);
        // each device's shard goes to its own slot of its full-size output (device order)
        const int rc = bn_pairing_many_dev(subs[k], d_p[k], d_q[k], n_per_dev, d_out[k] + k * n_per_dev, st[k]);
        if (rc) return mfail(c, rc, std::string("device shard: ") + bn_last_error(subs[k]));
    }
    Comms* cm = nullptr;
    if (int rc = comms_get(c, &cm)) return rc;
    cm->r.group_start();
    int e = 0;
    bool dev_ok = true;
    for (size_t k = 0; k < d && !e && dev_ok; ++k) {
        dev_ok = hipSetDevice(c->devices[k]) == hipSuccess;
        if (dev_ok)
            e = cm->r.all_gather(d_out[k] + k * n_per_dev, d_out[k], n_per_dev * sizeof(bn_gt), kNcclUint8,
                                 cm->comm[k], st[k]);
    }
    const int e2 = cm->r.group_end();  // always closes the group, also after an error above
    if (!dev_ok) return mfail(c, BN_ERR_HIP, "hipSetDevice");
    if (e || e2) return mfail(c, BN_ERR_HIP, std::string("ncclAllGather: ") + cm->r.error_string(e ? e : e2));
    return BN_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- host-buffer forms
int bn_multi_pairing_many(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out) {
    if (n && (!p || !q || !out)) return mfail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    return for_shards(c, n, [&](size_t k, size_t lo, size_t hi) {
        return bn_pairing_many(c->subs[k], p + lo, q + lo, hi - lo, out + lo);
    });
}
int bn_multi_final_exponentiation_many(bn_ctx* c, const bn_gt* f, size_t n, bn_gt* out, uint8_t* ok) {
    if (n && (!f || !out)) return mfail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    return for_shards(c, n, [&](size_t k, size_t lo, size_t hi) {
        return bn_final_exponentiation_many(c->subs[k], f + lo, hi - lo, out + lo, ok ? ok + lo : nullptr);
    });
}
int bn_multi_miller_loop_many(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out) {
    if (n && (!p || !q || !out)) return mfail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    return for_shards(c, n, [&](size_t k, size_t lo, size_t hi) {
        return bn_miller_loop_many(c->subs[k], p + lo, q + lo, hi - lo, out + lo);
    });
}
int bn_multi_g1_mul_many(bn_ctx* c, const bn_g1* p, const bn_fr* k_, size_t n, bn_g1* out) {
    if (n && (!p || !k_ || !out)) return mfail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    return for_shards(c, n, [&](size_t k, size_t lo, size_t hi) {
        return bn_g1_mul_many(c->subs[k], p + lo, k_ + lo, hi - lo, out + lo);
    });
}
int bn_multi_g2_mul_many(bn_ctx* c, const bn_g2* p, const bn_fr* k_, size_t n, bn_g2* out) {
    if (n && (!p || !k_ || !out)) return mfail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    return for_shards(c, n, [&](size_t k, size_t lo, size_t hi) {
        return bn_g2_mul_many(c->subs[k], p + lo, k_ + lo, hi - lo, out + lo);
    });
}

// per-device Miller products of the shards, multiplied on device 0 in device order
static int multi_miller_product(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, int mode, bn_gt* result,
                                bool* any) {
    const size_t d = c->subs.size();
    std::vector<bn_gt> part(d);
    std::vector<char> have(d, 0);
    int rc = for_shards(c, n, [&](size_t k, size_t lo, size_t hi) {
        have[k] = 1;
        return bn_internal_miller_product(c->subs[k], p + lo, q + lo, hi - lo, mode, &part[k]);
    });
    if (rc) return rc;
    bn_internal_gt_one(result);
    *any = false;
    for (size_t k = 0; k < d; ++k) {
        if (!have[k]) continue;
        if (!*any) {
            *result = part[k];
            *any = true;
            continue;
        }
        bn_gt prod;
        rc = bn_fq12_op_many(c->subs[0], BN_FQ12_MUL, result, &part[k], 1, &prod);
        if (rc) return mfail(c, rc, bn_last_error(c->subs[0]));
        *result = prod;
    }
    return BN_OK;
}

int bn_multi_pairing_batch(bn_ctx* c, const bn_g1* p, const bn_g2* q, size_t n, bn_gt* out) {
    if (!out || (n && (!p || !q))) return mfail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    if (n == 0) {  // mod.rs:922-924
        bn_internal_gt_one(out);
        return BN_OK;
    }
    bn_gt f;
    bool any = false;
    if (int rc = multi_miller_product(c, p, q, n, 0, &f, &any)) return rc;
    uint8_t ok = 1;
    const int rc = bn_final_exponentiation_many(c->subs[0], &f, 1, out, &ok);
    if (rc) return mfail(c, rc, bn_last_error(c->subs[0]));
    if (!ok) return mfail(c, BN_ERR_FE_ZERO, "miller loop cannot produce zero");
    return BN_OK;
}

int bn_multi_miller_loop_batch(bn_ctx* c, const bn_g2* q, const bn_g1* p, size_t n, bn_gt* out) {
    if (!out || (n && (!p || !q))) return mfail(c, BN_ERR_INVALID_ARGUMENT, "null buffer");
    bool any = false;
    if (n == 0) {
        bn_internal_gt_one(out);
        return BN_OK;
    }
    return multi_miller_product(c, p, q, n, 1, out, &any);
}

int bn_multi_destroy(bn_ctx* c) {
    if (c->comms) {
        Comms* cm = (Comms*)c->comms;
        for (void* m : cm->comm)
            if (m) cm->r.comm_destroy(m);
        delete cm;  // librccl stays loaded: RCCL keeps process-wide state
    }
    for (bn_ctx* d : c->subs) bn_ctx_destroy(d);
    c->subs.clear();
    delete c;
    return BN_OK;
}
