/*
 * pt_host.h -- C ABI of the host layer (libpt_host.so) for FFI callers (Python ctypes, tests).
 *
 * Wraps the C++ drop-in API of pathtracer_amd.hpp:
 *   pth_scene_*    SceneLoader.cpp:124-348 + BVH::build (BVH.cpp:5-228) + CpuHittable
 *                  (Hittable.cpp:115-190) without a GPU: parse, transform, build, inspect;
 *   pth_renderer_* the reference's Pathtracer class (Pathtracer.h:12-68) bound to one GPU (or a
 *                  row tile of the image), with loadScene() semantics for scene files.
 * Errors never terminate the process here: calls return PT_ERR_* (see pt_hip.h) and
 * pth_last_error() holds the message of the calling thread.
 */
#ifndef PT_HOST_H
#define PT_HOST_H

#include "pt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pth_scene pth_scene;
typedef struct pth_renderer pth_renderer;

PT_API const char *pth_last_error(void);

/* Scene file -> objects (file order), BVH (leaf size 4), camera for a width x height image,
 * textures decoded on the host (handle = load order, failures get handle 0 and no slot). */
PT_API int pth_scene_load(const char *path, uint32_t width, uint32_t height, pth_scene **out);
PT_API void pth_scene_free(pth_scene *scene);

/* Host-side wall time of the load: JSON parse + transforms (SceneLoader.cpp:124-348) and the SAH
 * BVH build (BVH.cpp:66-228; multi-threaded over independent subtrees, identical layout). */
PT_API int pth_scene_timing(const pth_scene *scene, double *parse_ms, double *bvh_ms);
PT_API uint32_t pth_scene_object_count(const pth_scene *scene);
PT_API uint32_t pth_scene_node_count(const pth_scene *scene);
PT_API uint32_t pth_scene_bvh_depth(const pth_scene *scene);
/* objects in file order as device records, plus their world AABBs (min xyz, max xyz) */
PT_API int pth_scene_objects(const pth_scene *scene, pt_hittable *objects, float *aabbs);
/* BVH nodes and the reordered primitives referenced by the leaves */
PT_API int pth_scene_bvh(const pth_scene *scene, pt_bvh_node *nodes, pt_hittable *prims);
PT_API int pth_scene_camera(const pth_scene *scene, pt_camera *camera);
PT_API uint32_t pth_scene_skybox(const pth_scene *scene);
PT_API uint32_t pth_scene_texture_count(const pth_scene *scene);
PT_API int pth_scene_texture_info(const pth_scene *scene, uint32_t handle, uint32_t *width, uint32_t *height);
PT_API int pth_scene_texture_data(const pth_scene *scene, uint32_t handle, float *rgba);

/* Camera ctor (Camera.inl:4-23, fovy in radians) and SceneLoader's degree conversion. */
PT_API int pth_camera_make(const float *position, const float *lookat, const float *up, float fovy_radians, float aspect,
                           pt_camera *out);

/* Camera::rotate / Camera::translate (Camera.inl:30-52) on a camera record, in place: the
 * interactive controls of main.cpp:330-376 (the reference resets the accumulation after either). */
PT_API int pth_camera_rotate(pt_camera *cam, float pitch, float yaw, float roll);
PT_API int pth_camera_translate(pt_camera *cam, float x, float y, float z);
PT_API float pth_radians(float degrees);

/* Pathtracer on `device`, covering rows y = row_offset + k * row_stride. */
PT_API int pth_renderer_create(uint32_t width, uint32_t height, int device, uint32_t row_offset, uint32_t row_stride,
                               pth_renderer **out);
/* Pathtracer on `device`, covering the row bands b = band_offset + k * band_stride of band_rows
 * rows each (pt_create_banded). */
PT_API int pth_renderer_create_banded(uint32_t width, uint32_t height, int device, uint32_t band_rows,
                                      uint32_t band_offset, uint32_t band_stride, pth_renderer **out);
/* Pathtracer over several GPUs of this process (pt_group_*): the image data calls return the full
 * image, gathered on devices[0] over RCCL; pth_renderer_gather_ms = wall time of the last gather. */
PT_API int pth_renderer_create_group(uint32_t width, uint32_t height, int ndev, const int *devices, uint32_t band_rows,
                                     pth_renderer **out);
PT_API float pth_renderer_gather_ms(const pth_renderer *r);
PT_API void pth_renderer_destroy(pth_renderer *r);
/* loadScene(pathtracer, params) for a scene file; fills the camera (aspect = width / height). */
PT_API int pth_renderer_load_scene(pth_renderer *r, const char *path, pt_camera *camera);
/* `chunks` x Pathtracer::render(camera, spp, ignore_history && first) in one launch. */
PT_API int pth_renderer_render(pth_renderer *r, const pt_camera *camera, uint32_t spp, uint32_t chunks, int ignore_history);
PT_API float pth_renderer_timing(const pth_renderer *r);
PT_API uint32_t pth_renderer_frames(const pth_renderer *r);
PT_API uint32_t pth_renderer_local_rows(const pth_renderer *r);
/* getHDRImageData / getImageData: borrowed pointers, valid until the next call */
PT_API const float *pth_renderer_hdr(pth_renderer *r);
PT_API const uint8_t *pth_renderer_image(pth_renderer *r);
PT_API pt_context *pth_renderer_context(pth_renderer *r);   /* devices[0]'s context for a group */
PT_API pt_group *pth_renderer_group(pth_renderer *r);       /* null unless multi-device */

/* Output files (main.cpp:180-199 semantics: rows flipped vertically when flip != 0). */
PT_API int pth_write_png(const char *path, uint32_t width, uint32_t height, const uint8_t *rgba, int flip);
PT_API int pth_write_hdr(const char *path, uint32_t width, uint32_t height, const float *rgba, int flip);

#ifdef __cplusplus
}
#endif

#endif /* PT_HOST_H */
