// sq_io.cpp -- binary checkpoint of a phi^4 slab (the
// reference's text start/end file, tauhost.c:91-173,562-581, is impractical at
// 10^7 sites).  A checkpoint is two files:
//   <path>        NumPy .npy v1.0, little-endian float32, shape (nz, Ly, Lx)
//                 (z slowest: exactly the slab's memory order), loadable by np.load;
//   <path>.json   {"format": "stochquant-phi4-slab", "version": 1, "dims": [Lx,Ly,Lz],
//                  "z0": ..., "nz": ..., "step": ..., "dtau": ..., "seed": ...}
// The Philox step counter is saved so a resumed run continues the same noise
// stream; Δτ is restored (the reference caps it at argv Δτ on resume, :131-136,
// which callers may apply).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "../../include/stochquant.h"
#include "sq_internal.h"

namespace {

int io_fail(const std::string &m) { return sq::set_error(SQ_E_ARG, m); }

bool write_npy(const char *path, const float *data, long long nz, long long ny, long long nx) {
    FILE *fp = fopen(path, "wb");
    if (!fp) return false;
    char dict[256];
    snprintf(dict, sizeof dict, "{'descr': '<f4', 'fortran_order': False, 'shape': (%lld, %lld, %lld), }",
             nz, ny, nx);
    std::string hdr(dict);
    const size_t pre = 10;  // magic(6) + version(2) + header length(2)
    size_t total = pre + hdr.size() + 1;
    const size_t pad = (64 - total % 64) % 64;
    hdr.append(pad, ' ');
    hdr.push_back('\n');
    const unsigned short hl = (unsigned short)hdr.size();
    const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
    bool ok = fwrite(magic, 1, 8, fp) == 8;
    const unsigned char hlb[2] = {(unsigned char)(hl & 0xFF), (unsigned char)(hl >> 8)};
    ok = ok && fwrite(hlb, 1, 2, fp) == 2;
    ok = ok && fwrite(hdr.data(), 1, hdr.size(), fp) == hdr.size();
    const size_t n = (size_t)(nz * ny * nx);
    ok = ok && fwrite(data, sizeof(float), n, fp) == n;
    return fclose(fp) == 0 && ok;
}

// Reads a float32 C-order .npy whose shape must equal want[3]; the header is
// checked before anything is allocated (a corrupt or foreign file fails here).
bool read_npy(const char *path, std::vector<float> &out, const long long want[3], std::string *why) {
    FILE *fp = fopen(path, "rb");
    if (!fp) {
        *why = "cannot open";
        return false;
    }
    unsigned char head[10];
    bool ok = fread(head, 1, 10, fp) == 10 && head[0] == 0x93 && memcmp(head + 1, "NUMPY", 5) == 0 &&
              head[6] == 1;
    std::string hdr;
    if (ok) {
        const size_t hl = head[8] | ((size_t)head[9] << 8);
        hdr.resize(hl);
        ok = fread(&hdr[0], 1, hl, fp) == hl;
    }
    ok = ok && hdr.find("'<f4'") != std::string::npos && hdr.find("'fortran_order': False") != std::string::npos;
    const size_t sp = ok ? hdr.find("'shape': (") : std::string::npos;
    long long shape[3] = {-1, -1, -1};
    ok = ok && sp != std::string::npos &&
         sscanf(hdr.c_str() + sp + 10, "%lld, %lld, %lld", &shape[0], &shape[1], &shape[2]) == 3;
    if (!ok) {
        *why = "not a float32 C-order 3-D .npy";
    } else if (shape[0] != want[0] || shape[1] != want[1] || shape[2] != want[2]) {
        *why = "shape (" + std::to_string(shape[0]) + ", " + std::to_string(shape[1]) + ", " +
               std::to_string(shape[2]) + ") does not match this slab (" + std::to_string(want[0]) + ", " +
               std::to_string(want[1]) + ", " + std::to_string(want[2]) + ")";
        ok = false;
    }
    if (ok) {
        const size_t n = (size_t)(want[0] * want[1] * want[2]);
        out.resize(n);
        ok = fread(out.data(), sizeof(float), n, fp) == n;
        if (!ok) *why = "truncated data";
    }
    fclose(fp);
    return ok;
}

bool read_text(const std::string &path, std::string *j) {
    FILE *fp = fopen(path.c_str(), "r");
    if (!fp) return false;
    char buf[512];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, fp)) > 0 && j->size() < (1u << 16)) j->append(buf, n);
    fclose(fp);
    return true;
}

bool json_dims(const std::string &j, long long d[3]) {
    const size_t p = j.find("\"dims\":");
    if (p == std::string::npos) return false;
    const size_t b = j.find('[', p);
    return b != std::string::npos && sscanf(j.c_str() + b + 1, "%lld , %lld , %lld", &d[0], &d[1], &d[2]) == 3;
}

long long json_int(const std::string &j, const char *key, bool *found) {
    const std::string k = std::string("\"") + key + "\":";
    const size_t p = j.find(k);
    *found = p != std::string::npos;
    return *found ? strtoll(j.c_str() + p + k.size(), nullptr, 10) : 0;
}

// Unsigned 64-bit fields (seed, step): strtoull, so values >= 2^63 round-trip
// (strtoll would saturate them to LLONG_MAX).
unsigned long long json_uint(const std::string &j, const char *key, bool *found) {
    const std::string k = std::string("\"") + key + "\":";
    const size_t p = j.find(k);
    *found = p != std::string::npos;
    return *found ? strtoull(j.c_str() + p + k.size(), nullptr, 10) : 0ull;
}

double json_dbl(const std::string &j, const char *key, bool *found) {
    const std::string k = std::string("\"") + key + "\":";
    const size_t p = j.find(k);
    *found = p != std::string::npos;
    return *found ? strtod(j.c_str() + p + k.size(), nullptr) : 0.0;
}

}  // namespace

extern "C" {

static int save_field(sq_ctx *ctx, const char *path) {
    int tile[4];
    if (sq_phi4_tile(ctx, tile) != SQ_OK) return io_fail("sq_save_field: PHI4 contexts only");
    long long nz = 0, z0 = 0;
    sq_slab(ctx, &nz, &z0);
    sq_params P;
    if (sq_get_params(ctx, &P) != SQ_OK) return io_fail("sq_get_params failed");
    std::vector<float> f((size_t)(nz * P.dims[1] * P.dims[0]));
    int rc = sq_download_field(ctx, f.data(), f.size());
    if (rc) return rc;
    if (!write_npy(path, f.data(), nz, P.dims[1], P.dims[0])) return io_fail(std::string("cannot write ") + path);
    unsigned long long step = 0;
    double dtau = 0;
    sq_get_step(ctx, &step);
    sq_get_dtau(ctx, &dtau);
    sq::FrameState fs{};
    if (sq::frame_state_get(ctx, &fs) != SQ_OK) return io_fail("frame state unavailable");
    const std::string jpath = std::string(path) + ".json";
    FILE *fp = fopen(jpath.c_str(), "w");
    if (!fp) return io_fail("cannot write " + jpath);
    // T and V exactly, as their IEEE bit patterns (a frame on an uploaded
    // field with inf seeds V = inf, which is not a JSON number); the decimal
    // values beside them are informative, null when not finite
    char tv[2][32];
    const float tvv[2] = {fs.T, fs.V};
    for (int i = 0; i < 2; ++i) {
        if (std::isfinite(tvv[i]))
            snprintf(tv[i], sizeof tv[i], "%.9g", (double)tvv[i]);
        else
            snprintf(tv[i], sizeof tv[i], "null");
    }
    uint32_t tb, vb;
    memcpy(&tb, &fs.T, sizeof tb);
    memcpy(&vb, &fs.V, sizeof vb);
    fprintf(fp,
            "{\"format\": \"stochquant-phi4-slab\", \"version\": 1, \"dims\": [%lld, %lld, %lld], "
            "\"z0\": %lld, \"nz\": %lld, \"step\": %llu, \"dtau\": %.17g, \"seed\": %llu, "
            "\"stab_init\": %d, \"stab_T\": %s, \"stab_V\": %s, \"stab_T_bits\": %u, \"stab_V_bits\": %u, "
            "\"stab_cnt\": %d}\n",
            P.dims[0], P.dims[1], P.dims[2], z0, nz, step, dtau, P.seed, fs.init, tv[0], tv[1], (unsigned)tb,
            (unsigned)vb, fs.stab_cnt);
    return fclose(fp) == 0 ? SQ_OK : io_fail("cannot write " + jpath);
}

int sq_save_field(sq_ctx *ctx, const char *path) {
    if (!ctx || !path) return io_fail("null argument");
    try {
        return save_field(ctx, path);
    } catch (const std::exception &e) {
        return io_fail(std::string("sq_save_field: ") + e.what());
    } catch (...) {
        return io_fail("sq_save_field: unexpected exception");
    }
}

// Validates everything (the .npy header against this slab, the metadata's
// dims / z0 / seed) before the device field is touched, so a failed load
// leaves the context's state as it was.
static int load_field(sq_ctx *ctx, const char *path, int restore_counters) {
    int tile[4];
    if (sq_phi4_tile(ctx, tile) != SQ_OK) return io_fail("sq_load_field: PHI4 contexts only");
    long long nz = 0, z0 = 0;
    sq_slab(ctx, &nz, &z0);
    sq_params P;
    if (sq_get_params(ctx, &P) != SQ_OK) return io_fail("sq_get_params failed");
    const std::string jpath = std::string(path) + ".json";
    std::string j;
    const bool have_meta = read_text(jpath, &j);
    if (restore_counters && !have_meta) return io_fail("cannot read " + jpath);
    unsigned long long step = 0;
    long long jz0 = 0, jnz = 0;
    double dtau = 0;
    // frame-control state (version-1 files written before round 3 lack it:
    // the heuristic then restarts from the field at the next frame)
    sq::FrameState fs{0.f, 0.f, 0, 0};
    bool have_fs = false;
    if (have_meta) {
        bool f1, f2, f3, f4, f5;
        step = json_uint(j, "step", &f1);
        dtau = json_dbl(j, "dtau", &f2);
        jz0 = json_int(j, "z0", &f3);
        jnz = json_int(j, "nz", &f4);
        const unsigned long long seed = json_uint(j, "seed", &f5);
        bool g1, g2, g3, g4;
        fs.init = (int)json_int(j, "stab_init", &g1);
        bool b2, b3;
        const unsigned long long tb = json_uint(j, "stab_T_bits", &b2);
        const unsigned long long vb = json_uint(j, "stab_V_bits", &b3);
        if (b2 && b3) {  // exact (files from round 4 on)
            const uint32_t t32 = (uint32_t)tb, v32 = (uint32_t)vb;
            memcpy(&fs.T, &t32, sizeof t32);
            memcpy(&fs.V, &v32, sizeof v32);
            g2 = g3 = true;
        } else {
            fs.T = (float)json_dbl(j, "stab_T", &g2);
            fs.V = (float)json_dbl(j, "stab_V", &g3);
        }
        fs.stab_cnt = (int)json_int(j, "stab_cnt", &g4);
        have_fs = g1 && g2 && g3 && g4;
        if (have_fs && fs.stab_cnt < 0) return io_fail("checkpoint stab_cnt must be >= 0");
        long long dims[3];
        if (!f1 || !f2 || !f3 || !f4 || !f5 || !json_dims(j, dims)) return io_fail("incomplete checkpoint metadata " + jpath);
        if (dims[0] != P.dims[0] || dims[1] != P.dims[1] || dims[2] != P.dims[2])
            return io_fail("checkpoint lattice dims do not match this context");
        if (jz0 != z0 || jnz != nz) return io_fail("checkpoint z0 / nz do not match this slab");
        // continuing the noise stream needs the same Philox key
        if (restore_counters && seed != P.seed) return io_fail("checkpoint seed does not match this context");
        if (restore_counters && !(dtau > 0)) return io_fail("checkpoint dtau must be > 0");
    }
    std::vector<float> f;
    const long long want[3] = {nz, P.dims[1], P.dims[0]};
    std::string why;
    if (!read_npy(path, f, want, &why)) return io_fail(std::string("cannot read field ") + path + ": " + why);
    int rc = sq_upload_field(ctx, f.data(), f.size());
    if (rc) return rc;
    if (restore_counters) {
        sq_set_step(ctx, step);
        sq_set_dtau(ctx, dtau);
        // the stability heuristic's T, V and the dtau controller's count carry
        // across frames: a resume continues them
        if (!have_fs) fs = sq::FrameState{0.f, 0.f, 0, 0};
        rc = sq::frame_state_set(ctx, fs);
        if (rc) return rc;
    }
    return SQ_OK;
}

int sq_load_field(sq_ctx *ctx, const char *path, int restore_counters) {
    if (!ctx || !path) return io_fail("null argument");
    try {  // no exception crosses the C ABI (std::bad_alloc on a huge slab, ...)
        return load_field(ctx, path, restore_counters);
    } catch (const std::exception &e) {
        return io_fail(std::string("sq_load_field: ") + e.what());
    } catch (...) {
        return io_fail("sq_load_field: unexpected exception");
    }
}

}  // extern "C"
