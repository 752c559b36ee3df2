/* render_scene.c -- a host program in plain C11 driving the drop-in boundary (include/rt_api.h,
 * include/rt_scene.h) with no Python and no torch: what a non-Python host of the reference's
 * device path would do in place of KernelLauncher (KernelLauncher.py:8-103).
 *
 *   render_scene SCENE.obj PARAMS.bin OUT_PREFIX
 *
 * SCENE.obj is parsed by the native importer (rt_obj_parse: FileManager.py:253-304 semantics) and
 * its BVH built by the native BVH.py builder (rt_bvh_build, bit-identical export).  The .ini side of
 * a scene (materials, camera, environment; FileManager.py:309-425, main.py:59-73) is the host's
 * business, as in the reference: PARAMS.bin carries it as little-endian words --
 *   int32 n_mat, float32 mat[6 n_mat], float32 cam[10], float32 env[5], int32 npix, int32 spp,
 *   int32 max_bounce, int32 ibl_w, int32 ibl_h, uint8 ibl_rgba[4 ibl_w ibl_h].
 * The program checks the scene on the host (rt_scene_check), renders it (rt_render, the
 * launch_Raytracing semantics), quantises it (rt_render_rgb8, FileManager.saveImg) and applies the
 * gamma kernel (rt_gamma, ImgProcessing.cl), and writes OUT_PREFIX.f32 (float32 RGB),
 * OUT_PREFIX.rgb8 and OUT_PREFIX.gamma.f32.  Exit status 0 on success. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_api.h"
#include "rt_scene.h"

static void* read_file(const char* path, long* size) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return NULL; }
    const long n = ftell(f);
    if (n < 0 || fseek(f, 0, SEEK_SET) != 0) { fclose(f); return NULL; }
    char* buf = (char*)malloc((size_t)n + 1);
    if (buf && fread(buf, 1, (size_t)n, f) != (size_t)n) { free(buf); buf = NULL; }
    fclose(f);
    if (buf) { buf[n] = 0; *size = n; }
    return buf;
}

static int write_file(const char* prefix, const char* suffix, const void* data, size_t bytes) {
    char path[4096];
    snprintf(path, sizeof path, "%s%s", prefix, suffix);
    FILE* f = fopen(path, "wb");
    if (!f) return 1;
    const int bad = fwrite(data, 1, bytes, f) != bytes;
    return fclose(f) != 0 || bad;
}

/* a cursor over PARAMS.bin */
typedef struct { const unsigned char* p; long left; } reader;
static int take(reader* r, void* dst, long bytes) {
    if (bytes < 0 || r->left < bytes) return 1;
    memcpy(dst, r->p, (size_t)bytes);
    r->p += bytes;
    r->left -= bytes;
    return 0;
}

#define FAIL(...) do { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); goto done; } while (0)

int main(int argc, char** argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: %s SCENE.obj PARAMS.bin OUT_PREFIX\n", argv[0]);
        return 2;
    }
    int rc = 1;
    rt_obj* obj = NULL;
    rt_ctx* ctx = NULL;
    char* text = NULL;
    unsigned char* params = NULL;
    float *vp = NULL, *vn = NULL, *vuv = NULL, *mat = NULL, *bvh = NULL, *out = NULL, *gam = NULL;
    int32_t* face = NULL;
    uint8_t *ibl = NULL, *out8 = NULL;

    long tlen = 0, plen = 0;
    text = (char*)read_file(argv[1], &tlen);
    if (!text) FAIL("cannot read %s", argv[1]);
    params = (unsigned char*)read_file(argv[2], &plen);
    if (!params) FAIL("cannot read %s", argv[2]);

    /* geometry: the native importer and BVH builder */
    if (rt_obj_parse(text, tlen, &obj) != RT_OK) FAIL("rt_obj_parse: %s", rt_obj_last_error());
    const int64_t nvp = rt_obj_size(obj, RT_OBJ_VP), nvn = rt_obj_size(obj, RT_OBJ_VN);
    const int64_t nvuv = rt_obj_size(obj, RT_OBJ_VUV), nface = rt_obj_size(obj, RT_OBJ_FACE);
    vp = (float*)malloc(sizeof(float) * (size_t)(nvp > 0 ? nvp : 1));
    vn = (float*)malloc(sizeof(float) * (size_t)(nvn > 0 ? nvn : 1));
    vuv = (float*)malloc(sizeof(float) * (size_t)(nvuv > 0 ? nvuv : 1));
    face = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nface > 0 ? nface : 1));
    if (!vp || !vn || !vuv || !face) FAIL("out of memory");
    if (rt_obj_copy(obj, vp, vn, vuv, face) != RT_OK) FAIL("rt_obj_copy: %s", rt_obj_last_error());
    const int64_t ntri = nface / 10;
    bvh = (float*)malloc(sizeof(float) * (size_t)(9 * (2 * ntri - 1 > 0 ? 2 * ntri - 1 : 1)));
    if (!bvh) FAIL("out of memory");
    int64_t nodes = 0;
    if (rt_bvh_build(face, nface, vp, nvp, bvh, &nodes) != RT_OK) FAIL("rt_bvh_build: %s", rt_last_error(NULL));

    /* the .ini side: materials, camera, environment, frame */
    reader r = {params, plen};
    int32_t nmat = 0, npix = 0, spp = 0, max_bounce = 0, iw = 0, ih = 0;
    float cam[10], env[5];
    if (take(&r, &nmat, 4) || nmat <= 0 || nmat > 1 << 20) FAIL("bad PARAMS: material count");
    mat = (float*)malloc(sizeof(float) * 6 * (size_t)nmat);
    if (!mat) FAIL("out of memory");
    if (take(&r, mat, 24L * nmat) || take(&r, cam, sizeof cam) || take(&r, env, sizeof env) || take(&r, &npix, 4) ||
        take(&r, &spp, 4) || take(&r, &max_bounce, 4) || take(&r, &iw, 4) || take(&r, &ih, 4))
        FAIL("bad PARAMS: truncated");
    if (npix <= 0 || iw <= 0 || ih <= 0 || (int64_t)iw * ih > (1 << 28)) FAIL("bad PARAMS: sizes");
    ibl = (uint8_t*)malloc(4 * (size_t)iw * (size_t)ih);
    if (!ibl || take(&r, ibl, 4L * iw * ih)) FAIL("bad PARAMS: IBL");

    /* host-side check first: the same validation rt_set_scene applies, no GPU */
    int64_t info[8];
    if (rt_scene_check(vp, nvp, vn, nvn, face, nface, mat, 6 * (int64_t)nmat, bvh, 9 * nodes, RT_BVH_SAH, info) != RT_OK)
        FAIL("rt_scene_check: %s", rt_scene_last_error());
    printf("scene: %lld triangles, %lld BVH nodes, FAST %s\n", (long long)info[0], (long long)info[1],
           info[7] ? "available" : "unavailable");

    /* the device path: KernelLauncher.__init__ + launch_Raytracing + launch_ImgProcessing */
    if (rt_device_count() < 1) FAIL("no HIP device");
    if (rt_create(1, NULL, &ctx) != RT_OK) FAIL("rt_create: %s", rt_last_error(NULL));
    if (rt_set_scene(ctx, vp, nvp, vn, nvn, vuv, nvuv, face, nface, mat, 6 * (int64_t)nmat, bvh, 9 * nodes) != RT_OK)
        FAIL("rt_set_scene: %s", rt_last_error(ctx));
    if (rt_set_env(ctx, ibl, iw, ih) != RT_OK) FAIL("rt_set_env: %s", rt_last_error(ctx));
    out = (float*)malloc(sizeof(float) * 3 * (size_t)npix);
    gam = (float*)malloc(sizeof(float) * 3 * (size_t)npix);
    out8 = (uint8_t*)malloc(3 * (size_t)npix);
    if (!out || !gam || !out8) FAIL("out of memory");
    if (rt_render(ctx, cam, env, npix, spp, max_bounce, out) != RT_OK) FAIL("rt_render: %s", rt_last_error(ctx));
    if (rt_render_rgb8(ctx, cam, env, npix, spp, max_bounce, 0, out8) != RT_OK)
        FAIL("rt_render_rgb8: %s", rt_last_error(ctx));
    if (rt_gamma(ctx, out, gam, 3 * (int64_t)npix) != RT_OK) FAIL("rt_gamma: %s", rt_last_error(ctx));
    /* a call the boundary must refuse, and say why */
    if (rt_set_option(ctx, "no_such_option", 1) == RT_OK) FAIL("an unknown option was accepted");
    printf("refused as expected: %s\n", rt_last_error(ctx));

    double sum = 0.0;
    for (int64_t k = 0; k < 3 * (int64_t)npix; ++k) sum += out[k];
    printf("rendered %d pixels at %d spp: mean %.6f\n", npix, spp, sum / (3.0 * npix));
    if (write_file(argv[3], ".f32", out, sizeof(float) * 3 * (size_t)npix) ||
        write_file(argv[3], ".rgb8", out8, 3 * (size_t)npix) ||
        write_file(argv[3], ".gamma.f32", gam, sizeof(float) * 3 * (size_t)npix))
        FAIL("cannot write %s.*", argv[3]);
    rc = 0;
done:
    if (ctx) rt_destroy(ctx);
    if (obj) rt_obj_free(obj);
    free(text); free(params); free(vp); free(vn); free(vuv); free(face); free(mat); free(bvh);
    free(ibl); free(out); free(gam); free(out8);
    return rc;
}
