// rs_capi.inl -- Reed-Solomon fragment coding entry points (dm_rs_*, include/deoss_merkle.h).
// Part of merkle_capi.hip (included at its end; shares dm_ctx, Dev, DevBuf and the error helpers).
//
// Mirrors github.com/klauspost/reedsolomon v1.12.4 (go.mod:65) as the cess-go-sdk uses it for
// DeOSS fragments (New(chain.DataShards = 4, chain.ParShards = 8), node/tracker.go:250,369):
//   New(data, parity)      -> dm_rs_create   (default Vandermonde-derived systematic matrix)
//   Encode(shards)         -> dm_rs_encode / dm_rs_encode_device_async
//   Reconstruct(shards)    -> dm_rs_reconstruct / dm_rs_reconstruct_device_async
//   Verify(shards)         -> dm_rs_verify
//   Split + Encode of one segment -> dm_rs_encode_buffer
// The GF(2^8) arithmetic below only builds the small coding tables; all shard bytes are coded
// by rs_code_kernel on the GPU (no CPU fallback).
#include "rs_kernels.hpp"

namespace {

struct Gf {
    uint8_t exp[510];
    uint8_t log[256];
    Gf() {
        unsigned x = 1;
        for (int i = 0; i < 255; i++) {
            exp[i] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11d;   // x^8 + x^4 + x^3 + x^2 + 1 (klauspost "29")
        }
        for (int i = 255; i < 510; i++) exp[i] = exp[i - 255];
        log[0] = 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
    uint8_t inv(uint8_t a) const { return exp[255 - log[a]]; }
    uint8_t pow(uint8_t a, int n) const { return n == 0 ? 1 : (a == 0 ? 0 : exp[(log[a] * n) % 255]); }
};

const Gf& gf() {
    static const Gf g;
    return g;
}

// Gauss-Jordan inverse of a k x k GF(2^8) matrix; false if singular.
bool gf_invert(const uint8_t* m, int k, uint8_t* out) {
    const Gf& g = gf();
    uint8_t w[dm::kRsMaxIn][2 * dm::kRsMaxIn];
    for (int r = 0; r < k; r++)
        for (int c = 0; c < k; c++) {
            w[r][c] = m[r * k + c];
            w[r][k + c] = (uint8_t)(r == c);
        }
    for (int c = 0; c < k; c++) {
        int p = c;
        while (p < k && w[p][c] == 0) p++;
        if (p == k) return false;
        if (p != c)
            for (int j = 0; j < 2 * k; j++) std::swap(w[p][j], w[c][j]);
        const uint8_t s = g.inv(w[c][c]);
        for (int j = 0; j < 2 * k; j++) w[c][j] = g.mul(w[c][j], s);
        for (int r = 0; r < k; r++) {
            if (r == c || w[r][c] == 0) continue;
            const uint8_t f = w[r][c];
            for (int j = 0; j < 2 * k; j++) w[r][j] ^= g.mul(f, w[c][j]);
        }
    }
    for (int r = 0; r < k; r++)
        for (int c = 0; c < k; c++) out[r * k + c] = w[r][k + c];
    return true;
}

// Lookup table of `rows` (nout x k, row-major): entry [j][x] byte i = rows[i][j] * x.
std::vector<uint64_t> rs_table(const uint8_t* rows, int nout, int k) {
    const Gf& g = gf();
    std::vector<uint64_t> t((size_t)k * 256, 0);
    for (int j = 0; j < k; j++)
        for (int x = 0; x < 256; x++) {
            uint64_t e = 0;
            for (int i = 0; i < nout; i++) e |= (uint64_t)g.mul(rows[i * k + j], (uint8_t)x) << (8 * i);
            t[(size_t)j * 256 + x] = e;
        }
    return t;
}

}  // namespace

namespace {

// One call lane's rs scratch: rs calls on different lanes of the first GPU run concurrently
// (dm_ctx call lanes), each with its own staging, so two uploads' FullProcessing overlap.
struct RsLane {
    DevBuf dec_tab;             // per reconstruct call
    DevBuf work;                // host-API shard staging, process parity, FullProcessing windows
    PinnedBuf fp_slot[4];       // dm_full_processing: file / parity slots (fullproc_capi.inl)
};

}  // namespace

struct dm_rs {
    dm_ctx* c = nullptr;
    int k = 0, m = 0;
    std::vector<uint8_t> mat;   // (k + m) x k
    DevBuf enc_tab;             // parity rows, k x 256 x 8 B (read-only after dm_rs_create)
    std::vector<RsLane> ln;     // one per call lane of the context's first GPU
};

namespace {

// Lane of the context's first GPU (where an rs lives) for an rs call, counted in its load like
// pick_device (the caller's CallLock(..., kReserved) releases it).
int rs_lane(dm_ctx* c) {
    std::lock_guard<std::mutex> lk(c->route_mu);
    return choose_lane(c, 0, 0);
}

// The rs scratch of the lane d belongs to (d is one of r->c->devs, on the first GPU).
RsLane& rs_ln(dm_rs* r, const Dev& d) {
    return r->ln[(size_t)(&d - r->c->devs.data()) / (size_t)r->c->nphys];
}

void launch_rs(Dev& d, hipStream_t s, int k, const dm::RsArgs& a) {
    const uint64_t units = a.units_per_seg;
    const uint64_t target = 8ull * (uint64_t)d.cus;   // workgroups in flight
    const uint32_t gy = (uint32_t)std::min<uint64_t>({a.nseg, 65535ull, target});
    const uint32_t gx = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(units, dm::kRsThreads),
                                                                           ceil_div(target, gy)));
    const dim3 grid(gx, gy), block(dm::kRsThreads);
    switch (k) {
        case 1: hipLaunchKernelGGL(dm::rs_code_kernel<1>, grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL(dm::rs_code_kernel<2>, grid, block, 0, s, a); break;
        case 3: hipLaunchKernelGGL(dm::rs_code_kernel<3>, grid, block, 0, s, a); break;
        case 4: hipLaunchKernelGGL(dm::rs_code_kernel<4>, grid, block, 0, s, a); break;
        case 5: hipLaunchKernelGGL(dm::rs_code_kernel<5>, grid, block, 0, s, a); break;
        case 6: hipLaunchKernelGGL(dm::rs_code_kernel<6>, grid, block, 0, s, a); break;
        case 7: hipLaunchKernelGGL(dm::rs_code_kernel<7>, grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL(dm::rs_code_kernel<8>, grid, block, 0, s, a); break;
    }
}

// Coding rows that rebuild the missing shards from the first k present ones (klauspost
// Reconstruct: the first `data` valid shards in index order; missing data rows come from the
// inverse of their sub-matrix, missing parity rows = parity row x that inverse).
int rs_decode_plan(dm_rs* r, const uint8_t* present, int* valid, int* missing, int* nmiss, std::vector<uint8_t>& rows) {
    dm_ctx* c = r->c;
    const int k = r->k, total = r->k + r->m;
    int nv = 0;
    *nmiss = 0;
    for (int i = 0; i < total; i++) {
        if (present[i]) {
            if (nv < k) valid[nv++] = i;
        } else {
            missing[(*nmiss)++] = i;
        }
    }
    if (nv < k) return fail(c, DM_ERR_INVALID, "too few shards given (%d of %d needed)", nv, k);
    uint8_t sub[dm::kRsMaxIn * dm::kRsMaxIn], inv[dm::kRsMaxIn * dm::kRsMaxIn];
    for (int i = 0; i < k; i++) std::memcpy(sub + i * k, r->mat.data() + valid[i] * k, (size_t)k);
    if (!gf_invert(sub, k, inv)) return fail(c, DM_ERR_INVALID, "singular decode matrix");
    const Gf& g = gf();
    rows.assign((size_t)*nmiss * k, 0);
    for (int t = 0; t < *nmiss; t++) {
        const uint8_t* mrow = r->mat.data() + missing[t] * k;   // output = mrow x data = mrow x inv x valid
        for (int j = 0; j < k; j++) {
            uint8_t acc = 0;
            for (int q = 0; q < k; q++) acc ^= g.mul(mrow[q], inv[q * k + j]);
            rows[(size_t)t * k + j] = acc;
        }
    }
    return DM_OK;
}

int rs_reconstruct_dev(dm_rs* r, Dev& d, hipStream_t s, uint8_t* const* shards, const uint8_t* present,
                       uint64_t pitch, uint64_t nbytes_units) {
    dm_ctx* c = r->c;
    int valid[dm::kRsMaxIn + dm::kRsMaxOut], missing[dm::kRsMaxIn + dm::kRsMaxOut], nmiss = 0;
    std::vector<uint8_t> rows;
    RC_TRY(rs_decode_plan(r, present, valid, missing, &nmiss, rows));
    if (nmiss == 0) return DM_OK;
    const std::vector<uint64_t> tab = rs_table(rows.data(), nmiss, r->k);
    RC_TRY(tables_begin(c, d, tab.size() * 8));
    RsLane& L = rs_ln(r, d);
    RC_TRY(upload(c, d, s, L.dec_tab, tab.data(), tab.size() * 8));
    dm::RsArgs a{};
    for (int j = 0; j < r->k; j++) a.in[j] = shards[valid[j]];
    for (int t = 0; t < nmiss; t++) a.out[t] = shards[missing[t]];
    a.in_seg_stride = a.out_seg_stride = pitch;
    a.units_per_seg = nbytes_units;
    a.nseg = 1;
    a.table = static_cast<const uint2*>(L.dec_tab.p);
    a.nout = (uint32_t)nmiss;
    launch_rs(d, s, r->k, a);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

}  // namespace

extern "C" {

int dm_rs_create(dm_ctx* ctx, int data_shards, int parity_shards, dm_rs** out) {
    if (!ctx || !out) return bad_arg();
    *out = nullptr;
    CallLock lk(ctx, 0);
    dm_ctx* c = ctx;
    if (data_shards < 1 || data_shards > dm::kRsMaxIn || parity_shards < 1 || parity_shards > dm::kRsMaxOut)
        return fail(c, DM_ERR_INVALID, "shard counts: 1 <= data <= %d, 1 <= parity <= %d", dm::kRsMaxIn,
                    dm::kRsMaxOut);
    dm_rs* r = new (std::nothrow) dm_rs();
    if (!r) return fail(c, DM_ERR_NOMEM, "dm_rs_create: out of host memory");
    r->c = ctx;
    r->k = data_shards;
    r->m = parity_shards;
    const int k = data_shards, total = data_shards + parity_shards;
    // buildMatrix: vandermonde(total, k) x inverse(top k x k)
    const Gf& g = gf();
    std::vector<uint8_t> vm((size_t)total * k);
    for (int i = 0; i < total; i++)
        for (int j = 0; j < k; j++) vm[(size_t)i * k + j] = g.pow((uint8_t)i, j);
    uint8_t inv[dm::kRsMaxIn * dm::kRsMaxIn];
    if (!gf_invert(vm.data(), k, inv)) {
        delete r;
        return fail(c, DM_ERR_INVALID, "singular Vandermonde top");
    }
    r->mat.assign((size_t)total * k, 0);
    for (int i = 0; i < total; i++)
        for (int j = 0; j < k; j++) {
            uint8_t acc = 0;
            for (int t = 0; t < k; t++) acc ^= g.mul(vm[(size_t)i * k + t], inv[t * k + j]);
            r->mat[(size_t)i * k + j] = acc;
        }
    const std::vector<uint64_t> tab = rs_table(r->mat.data() + (size_t)k * k, parity_shards, k);
    Dev& d = ctx->devs[0];
    r->ln.resize((size_t)ctx->lanes);
    r->enc_tab.rp = &ctx->reaper;
    r->enc_tab.dev = d.id;
    for (RsLane& L : r->ln)
        for (DevBuf* b : {&L.dec_tab, &L.work}) {
            b->rp = &ctx->reaper;   // growth (work: FullProcessing windows) never synchronises the device
            b->dev = d.id;
        }
    hipError_t e = hipSetDevice(d.id);
    if (e == hipSuccess) e = r->enc_tab.ensure(tab.size() * 8);
    // on the first lane's copy stream (non-blocking), not hipMemcpy's null stream: that one would
    // wait for every lane's queued chains on this GPU (their compute streams order with it)
    if (e == hipSuccess) e = hipMemcpyAsync(r->enc_tab.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, d.copy);
    if (e == hipSuccess) e = hipStreamSynchronize(d.copy);
    if (e != hipSuccess) {
        r->enc_tab.release();
        delete r;
        return fail(c, DM_ERR_HIP, "dm_rs_create: %s", hipGetErrorString(e));
    }
    *out = r;
    return DM_OK;
}

void dm_rs_destroy(dm_rs* r) {
    if (!r) return;
    {
        RangeLock lk(r->c);   // after every call in flight on any lane
        (void)hipSetDevice(r->c->devs[0].id);
        (void)hipDeviceSynchronize();
        r->enc_tab.release();
        for (RsLane& L : r->ln) {
            L.dec_tab.release();
            L.work.release();
            for (auto& b : L.fp_slot) b.release();
        }
    }
    delete r;
}

int dm_rs_matrix(dm_rs* r, uint8_t* out) {
    if (!r || !out) return bad_arg();
    std::memcpy(out, r->mat.data(), r->mat.size());
    return DM_OK;
}

int dm_rs_encode_device_async(dm_rs* r, const void* data, uint64_t data_stride, void* parity, uint64_t parity_stride,
                              uint64_t shard, uint64_t nseg, void* stream) {
    if (!r) return bad_arg();
    dm_ctx* c = r->c;
    const int g = rs_lane(c);
    CallLock lk(c, g, kReserved);
    if (!data || !parity || nseg == 0 || shard == 0 || shard % 16 || data_stride % 16 || parity_stride % 16 ||
        !is_aligned16(data) || !is_aligned16(parity))
        return fail(c, DM_ERR_INVALID, "dm_rs_encode_device_async: need 16-byte aligned shards, strides and sizes");
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    dm::RsArgs a{};
    for (int j = 0; j < r->k; j++) a.in[j] = static_cast<const uint8_t*>(data) + (uint64_t)j * shard;
    for (int i = 0; i < r->m; i++) a.out[i] = static_cast<uint8_t*>(parity) + (uint64_t)i * shard;
    a.in_seg_stride = data_stride;
    a.out_seg_stride = parity_stride;
    a.units_per_seg = shard / 16;
    a.nseg = nseg;
    a.table = static_cast<const uint2*>(r->enc_tab.p);
    a.nout = (uint32_t)r->m;
    hipEvent_t* tr = timing_record(c, d);
    if (tr) HIP_TRY(hipEventRecord(tr[0], s));
    launch_rs(d, s, r->k, a);
    HIP_TRY(hipGetLastError());
    if (tr) {
        HIP_TRY(hipEventRecord(tr[1], s));
        HIP_TRY(hipEventRecord(tr[2], s));
    }
    return DM_OK;
}

int dm_rs_reconstruct_device_async(dm_rs* r, void* const* shards, const uint8_t* present, uint64_t shard,
                                   void* stream) {
    if (!r) return bad_arg();
    dm_ctx* c = r->c;
    const int g = rs_lane(c);
    CallLock lk(c, g, kReserved);
    if (!shards || !present || shard == 0 || shard % 16)
        return fail(c, DM_ERR_INVALID, "dm_rs_reconstruct_device_async: shard bytes must be a multiple of 16");
    for (int i = 0; i < r->k + r->m; i++)
        if (!shards[i] || !is_aligned16(shards[i]))
            return fail(c, DM_ERR_INVALID, "dm_rs_reconstruct_device_async: shard %d null or not 16-byte aligned", i);
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    return rs_reconstruct_dev(r, d, s, reinterpret_cast<uint8_t* const*>(shards), present, shard, shard / 16);
}

// Host shards: staged in one device buffer at a 16-byte pitch (padding positions are coded too
// and never copied back; positions are independent).
int dm_rs_encode(dm_rs* r, const void* const* data, void* const* parity, uint64_t shard) {
    if (!r) return bad_arg();
    dm_ctx* c = r->c;
    const int g = rs_lane(c);
    CallLock lk(c, g, kReserved);
    if (!data || !parity || shard == 0) return fail(c, DM_ERR_INVALID, "dm_rs_encode: null shards or zero size");
    for (int j = 0; j < r->k; j++)
        if (!data[j]) return fail(c, DM_ERR_INVALID, "dm_rs_encode: data shard %d is null", j);
    for (int i = 0; i < r->m; i++)
        if (!parity[i]) return fail(c, DM_ERR_INVALID, "dm_rs_encode: parity shard %d is null", i);
    Dev& d = c->devs[g];
    DevBuf& work = rs_ln(r, d).work;
    hipStream_t s = d.stream;
    RC_TRY(begin_call(c, d, s));
    const uint64_t pitch = round_up(shard, 16);
    const int total = r->k + r->m;
    HIP_TRY(work.ensure(pitch * total));
    for (int j = 0; j < r->k; j++)
        HIP_TRY(hipMemcpyAsync(work.u8() + j * pitch, data[j], shard, hipMemcpyHostToDevice, s));
    dm::RsArgs a{};
    for (int j = 0; j < r->k; j++) a.in[j] = work.u8() + j * pitch;
    for (int i = 0; i < r->m; i++) a.out[i] = work.u8() + (r->k + i) * pitch;
    a.in_seg_stride = a.out_seg_stride = 0;
    a.units_per_seg = pitch / 16;
    a.nseg = 1;
    a.table = static_cast<const uint2*>(r->enc_tab.p);
    a.nout = (uint32_t)r->m;
    launch_rs(d, s, r->k, a);
    HIP_TRY(hipGetLastError());
    for (int i = 0; i < r->m; i++)
        HIP_TRY(hipMemcpyAsync(parity[i], work.u8() + (r->k + i) * pitch, shard, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return DM_OK;
}

int dm_rs_encode_buffer(dm_rs* r, const void* host, uint64_t len, void* out, uint64_t* per_shard) {
    if (!r) return bad_arg();
    if (!per_shard || !out || (!host && len)) return fail(r->c, DM_ERR_INVALID, "dm_rs_encode_buffer: null argument");
    if (len == 0) return fail(r->c, DM_ERR_EMPTY, "Empty data");   // klauspost ErrShortData
    const uint64_t per = ceil_div(len, (uint64_t)r->k);
    *per_shard = per;
    uint8_t* o = static_cast<uint8_t*>(out);
    // Split: data shards are the buffer in order, the last one zero-padded
    std::memcpy(o, host, len);
    std::memset(o + len, 0, per * r->k - len);
    std::vector<const void*> dp(r->k);
    std::vector<void*> pp(r->m);
    for (int j = 0; j < r->k; j++) dp[j] = o + j * per;
    for (int i = 0; i < r->m; i++) pp[i] = o + (r->k + i) * per;
    return dm_rs_encode(r, dp.data(), pp.data(), per);
}

int dm_rs_reconstruct(dm_rs* r, void* const* shards, const uint8_t* present, uint64_t shard) {
    if (!r) return bad_arg();
    dm_ctx* c = r->c;
    const int g = rs_lane(c);
    CallLock lk(c, g, kReserved);
    const int total = r->k + r->m;
    if (!shards || !present || shard == 0) return fail(c, DM_ERR_INVALID, "dm_rs_reconstruct: bad arguments");
    for (int i = 0; i < total; i++)
        if (!shards[i]) return fail(c, DM_ERR_INVALID, "dm_rs_reconstruct: shard %d is null", i);
    int nv = 0;
    for (int i = 0; i < total; i++) nv += present[i] != 0;
    if (nv == total) return DM_OK;
    if (nv < r->k) return fail(c, DM_ERR_INVALID, "too few shards given (%d of %d needed)", nv, r->k);
    Dev& d = c->devs[g];
    DevBuf& work = rs_ln(r, d).work;
    hipStream_t s = d.stream;
    RC_TRY(begin_call(c, d, s));
    const uint64_t pitch = round_up(shard, 16);
    HIP_TRY(work.ensure(pitch * total));
    std::vector<uint8_t*> dev(total);
    for (int i = 0; i < total; i++) {
        dev[i] = work.u8() + i * pitch;
        if (present[i]) HIP_TRY(hipMemcpyAsync(dev[i], shards[i], shard, hipMemcpyHostToDevice, s));
    }
    RC_TRY(rs_reconstruct_dev(r, d, s, dev.data(), present, pitch, pitch / 16));
    for (int i = 0; i < total; i++)
        if (!present[i]) HIP_TRY(hipMemcpyAsync(shards[i], dev[i], shard, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return DM_OK;
}

int dm_rs_verify(dm_rs* r, const void* const* shards, uint64_t shard, int* ok) {
    if (!r || !ok) return bad_arg();
    *ok = 0;
    if (!shards || shard == 0) return fail(r->c, DM_ERR_INVALID, "dm_rs_verify: bad arguments");
    std::vector<std::vector<uint8_t>> mine(r->m, std::vector<uint8_t>(shard));
    std::vector<void*> pp(r->m);
    for (int i = 0; i < r->m; i++) pp[i] = mine[i].data();
    RC_TRY(dm_rs_encode(r, shards, pp.data(), shard));
    for (int i = 0; i < r->m; i++) {
        if (!shards[r->k + i]) return fail(r->c, DM_ERR_INVALID, "dm_rs_verify: parity shard %d is null", i);
        if (std::memcmp(mine[i].data(), shards[r->k + i], shard) != 0) return DM_OK;
    }
    *ok = 1;
    return DM_OK;
}

}  // extern "C"
