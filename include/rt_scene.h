/* rt_scene.h -- native scene import with the reference importer's semantics
 * (SURVEY.md 8(f) row 2).  Host-only, no GPU needed.
 *
 *   rt_obj_parse   <- FileManager.Scene's OBJ read (FileManager.py:253-304):
 *                     V_p / V_n / V_uv from v / vn / vt lines, faceData
 *                     [mat, uv0..2, n0..2, p0..2] (0-based) from 'f' lines after
 *                     the first "usemtl", material counter from 'u' lines.
 *
 * Usage: rt_obj_parse(text, len, &obj); n = rt_obj_size(obj, RT_OBJ_VP); ...;
 * rt_obj_copy(obj, vp, vn, vuv, face); rt_obj_free(obj).  On failure (a line
 * the reference's parser would raise on) the call returns non-zero and
 * rt_obj_last_error() describes it.
 *
 *   rt_scene_check <- the checks and repacking rt_set_scene (rt_api.h) applies to
 *                     the arrays KernelLauncher.launch_Raytracing uploads
 *                     (KernelLauncher.py:38-72), run on the host alone: no
 *                     context, no GPU.  Returns RT_OK or the RT_ERR_* code
 *                     rt_set_scene would return; rt_scene_last_error() says why
 *                     (also, with RT_OK, why the FAST layouts are unavailable).
 *                     info (may be NULL): triangles, BVH2 nodes, BVH2 stack
 *                     depth, 4-wide nodes, 4-wide depth, brute-force records,
 *                     distinct leaf boxes, FAST available (0/1). */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_obj rt_obj;

enum rt_obj_array {
    RT_OBJ_VP = 0,        /* float32 count of V_p (3 per vertex) */
    RT_OBJ_VN = 1,        /* float32 count of V_n */
    RT_OBJ_VUV = 2,       /* float32 count of V_uv (2 per texture coordinate) */
    RT_OBJ_FACE = 3,      /* int32 count of faceData (10 per triangle) */
    RT_OBJ_MATERIALS = 4  /* the reference's matCounter */
};

int rt_obj_parse(const char* text, int64_t len, rt_obj** out);
int64_t rt_obj_size(const rt_obj* obj, int what);
/* Copies into caller arrays sized by rt_obj_size; any pointer may be NULL. */
int rt_obj_copy(const rt_obj* obj, float* vp, float* vn, float* vuv, int32_t* face);
void rt_obj_free(rt_obj* obj);
const char* rt_obj_last_error(void);

int rt_scene_check(const float* vp, int64_t nvp, const float* vn, int64_t nvn, const int32_t* face, int64_t nface,
                   const float* mat, int64_t nmat, const float* bvh9, int64_t nbvh, int layout, int64_t info[8]);
const char* rt_scene_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_SCENE_H */
