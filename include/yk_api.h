/*
 * yk_api.h -- C-ABI boundary of the MI355X ray-scene intersection and
 * path-integrator hot path (libyk.so).
 *
 * Replaces, behind the reference's own plugin API, these reference entry points
 * (reference = inferrna/Core, TheBounty 0.1.6):
 *   scene_t::startTriMesh/addVertex/addTriangle/endTriMesh  scene.cc:265-320,520-625
 *   scene_t::update (prim gather + triKdTree_t build)        scene.cc:748-850
 *   scene_t::intersect  -> triKdTree_t::Intersect            scene.cc:852-879, kdtree.cc:675-817
 *   scene_t::isShadowed -> triKdTree_t::IntersectS           scene.cc:881-902, kdtree.cc:820-947
 *   tiledIntegrator_t::render/renderPass/renderTile          integrator.cc:132-339
 *   pathIntegrator_t::integrate                              pathtracer.cc:134-333
 *   directLighting_t::integrate                              directlight.cc:112-182
 *   imageFilm_t::addSample / flush                           imagefilm.cc:383-511
 * The C++ plugin (plugin/yk_pathtrace_plugin.cc) binds these from inside a
 * tiledIntegrator_t subclass registered as "pathtracing"/"directlighting".
 *
 * Conventions: every function returns 0 (YK_OK) or a YK_ERR_* code; the text
 * of the last error of the calling thread is yk_last_error(). No C++ exception
 * and no HIP error crosses this boundary. Pointers named d_* are device (HBM)
 * pointers on the device the yk_device was opened on; all others are host.
 */
#ifndef YK_API_H
#define YK_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YK_OK 0
#define YK_ERR_ARG 1
#define YK_ERR_STATE 2
#define YK_ERR_HIP 3
#define YK_ERR_UNSUPPORTED 4
#define YK_ERR_ALLOC 5
#define YK_ERR_INTERNAL 6
#define YK_ERR_ABORTED 7 /* the abort callback asked to stop: the film holds the finished batches */

/* ---- scene description (POD mirrors of the reference paraMap_t params) ---- */

enum { YK_MAT_SHINYDIFFUSE = 0, YK_MAT_LIGHT = 1 };
typedef struct yk_material {
  int32_t type;           /* YK_MAT_*                                               */
  float color[3];         /* "color"  shinydiffuse.cc:474,483 / simple.cc:82        */
  float diffuse_reflect;  /* "diffuse_reflect" (shinydiffusemat, default 1)         */
  float emit;             /* "emit" (shinydiffusemat, default 0)                    */
  float power;            /* "power" (light_mat, default 1)                         */
  int32_t double_sided;   /* "double_sided" (light_mat, default 0)                  */
  /* shinydiffusemat specular / transmissive parameters (shinydiffuse.cc:474-503;
   * reference defaults in brackets -- a zero-initialised struct must set them) */
  float mirror_color[3];  /* "mirror_color" [1,1,1]                                 */
  float specular_reflect; /* "specular_reflect" [0]: mirror strength                */
  float transparency;     /* "transparency" [0]                                     */
  float translucency;     /* "translucency" [0]                                     */
  float transmit_filter;  /* "transmit_filter" [1]                                  */
  int32_t fresnel_effect; /* "fresnel_effect" [0]                                   */
  double ior;             /* "IOR" [1.33] (parsed as double; mIOR_Squared = IOR*IOR) */
  /* "diffuse_brdf" (shinydiffuse.cc:505-514): YK_BRDF_LAMBERT [default] or
   * YK_BRDF_OREN_NAYAR ("oren_nayar"), whose roughness is "sigma" [0.1,
   * parsed as double; a zero-initialised struct must set it]:
   * initOrenNayar(sigma), shinydiffuse.cc:170-176 */
  int32_t diffuse_brdf;
  double sigma;
} yk_material;
enum { YK_BRDF_LAMBERT = 0, YK_BRDF_OREN_NAYAR = 1 };

enum { YK_LIGHT_AREA = 0, YK_LIGHT_POINT = 1, YK_LIGHT_DIRECTIONAL = 2 };
typedef struct yk_light {
  int32_t type;
  /* area: areaLight_t::factory, arealight.cc:171-192 */
  float corner[3], point1[3], point2[3];
  float color[3];
  float power;
  int32_t samples;
  /* point: pointLight_t::factory (pointlight.cc:129-139), position = from;
   * directional: directionalLight_t::factory (directional.cc:139-165):
   * direction, and from/radius when infinite == 0 */
  float from[3];
  float direction[3];
  float radius;
  int32_t infinite;
} yk_light;

/* perspectiveCam_t bokeh shapes and bias (perspectiveCamera.h:33-34) */
enum { YK_BOKEH_DISK1 = 0, YK_BOKEH_DISK2 = 1, YK_BOKEH_TRI = 3, YK_BOKEH_SQR = 4, YK_BOKEH_PENTA = 5,
       YK_BOKEH_HEXA = 6, YK_BOKEH_RING = 7 };
enum { YK_BOKEH_BIAS_NONE = 0, YK_BOKEH_BIAS_CENTER = 1, YK_BOKEH_BIAS_EDGE = 2 };
typedef struct yk_camera { /* perspectiveCam_t::factory, perspectiveCamera.cc:191-232 */
  float from[3], to[3], up[3];
  int32_t resx, resy;
  float focal, aspect_ratio, near_clip, far_clip;
  /* depth of field: "aperture" [0 = pinhole], "dof_distance", "bokeh_type",
   * "bokeh_bias", "bokeh_rotation" (degrees) */
  float aperture, dof_distance;
  int32_t bokeh_type, bokeh_bias;
  float bokeh_rotation;
} yk_camera;

enum { YK_INTEGRATOR_DIRECT = 0, YK_INTEGRATOR_PATH = 1, YK_INTEGRATOR_PHOTON = 2 };
enum { YK_FILTER_BOX = 0, YK_FILTER_MITCHELL = 1, YK_FILTER_GAUSS = 2, YK_FILTER_LANCZOS = 3 };
/* pathtracing "caustic_type" (pathtracer.cc:367-385): photon / both build a
 * caustic photon map in preprocess (mcIntegrator_t::createCausticMap,
 * mcintegrator.cc:197-377) from params.photon: caustic_photons ("photons"),
 * caustic_mix ("caustic_mix"), caustic_radius ("caustic_radius") and bounces
 * (= "caustic_depth", default 10 there); yk_photon_build builds it. */
enum { YK_CAUSTIC_NONE = 0, YK_CAUSTIC_PATH = 1, YK_CAUSTIC_PHOTON = 2, YK_CAUSTIC_BOTH = 3 };

/* photonIntegrator_t parameters (photonintegr.cc:884-960 factory; defaults
 * in brackets, set by yk_render_params_default). */
typedef struct yk_photon_params {
  int32_t photons;         /* "photons" [100000]: diffuse photons shot                */
  int32_t caustic_photons; /* "cPhotons" [500000]                                     */
  float diffuse_radius;    /* "diffuseRadius" [0.1]                                   */
  float caustic_radius;    /* "causticRadius" [0.01]                                  */
  int32_t search;          /* "search" [50]: nDiffuseSearch                           */
  int32_t caustic_mix;     /* "caustic_mix" [= search]: nCausSearch                   */
  int32_t bounces;         /* "bounces" [5]: maxBounces of the photon paths           */
  int32_t final_gather;    /* "finalGather" [1]                                       */
  int32_t fg_samples;      /* "fg_samples" [32]: nPaths                               */
  int32_t fg_bounces;      /* "fg_bounces" [2]: gatherBounces                         */
  float fg_min_pathlen;    /* "fg_min_pathlen" [= diffuseRadius]: gatherDist          */
  int32_t show_map;        /* "show_map" [0]                                          */
  int32_t seed;            /* the global ourRandom() state (myseed, vector3d.cc:185)
                              when preprocess() starts [123212]                       */
} yk_photon_params;

typedef struct yk_render_params {
  int32_t integrator;     /* YK_INTEGRATOR_*                                         */
  int32_t raydepth;       /* "raydepth"                                              */
  int32_t path_samples;   /* "path_samples" (pathtracing)                            */
  int32_t bounces;        /* "bounces" (pathtracing)                                 */
  int32_t caustic_type;   /* "caustic_type": YK_CAUSTIC_NONE or YK_CAUSTIC_PATH      */
  int32_t width, height;  /* render area ("width"/"height")                          */
  int32_t xstart, ystart; /* crop offset ("xstart"/"ystart")                         */
  int32_t aa_samples;     /* "AA_minsamples"                                         */
  int32_t aa_passes;      /* "AA_passes" (> 1: adaptive passes, single shard only)   */
  int32_t filter;         /* YK_FILTER_*                                             */
  float aa_pixelwidth;    /* "AA_pixelwidth"                                         */
  int32_t tile_size;      /* "tile_size"                                             */
  int32_t transp_background; /* "bg_transp" (default 1)                             */
  int32_t aa_inc_samples; /* "AA_inc_samples": samples per pass after the first (<= 0:
                             aa_samples, scene_t::setAntialiasing scene.cc:736-742)    */
  float aa_threshold;     /* "AA_threshold" (default 0.05): adaptive resampling     */
  yk_photon_params photon; /* integrator == YK_INTEGRATOR_PHOTON                   */
  int32_t transp_shadows;  /* "transpShad" [0]: shadow rays pass transparent materials,
                              scene_t::isShadowed(.., maxDepth, filt) / IntersectTS    */
  int32_t shadow_depth;    /* "shadowDepth" [5]: transparent surfaces a shadow ray may
                              cross (mcIntegrator_t::sDepth)                           */
  float filter_width;      /* imageFilm_t::filterw as the film holds it (> 0), taking
                              precedence over aa_pixelwidth; 0: derived from
                              aa_pixelwidth as imagefilm.cc:143-150 does [0]            */
  /* The order in which the film hands out its tiles (imageFilm_t::nextArea
   * over its imageSpliter_t, imagefilm.cc:190-195,291-304): tile_order_len
   * tile indices ty * ntx + tx, a permutation of all of the render area's
   * tiles; NULL / 0: row-major ("tiles_order" "linear", imagesplitter.cc:
   * 29-45). For "random" (std::random_shuffle, imagesplitter.cc:48) a plugin
   * reads the live film's splitter; yk_tile_order_random computes it for a
   * given rand() seed. Samples are splatted in this order (single-thread
   * reference order); a shard renders the listed tiles t with
   * t % nshards == shard, in list order. [NULL, 0]                           */
  const int32_t* tile_order;
  int32_t tile_order_len;
} yk_render_params;
enum { YK_TILES_LINEAR = 0, YK_TILES_RANDOM = 1 };

/* one ray, 32 bytes: ray_t (ray.h:26-49) without time */
typedef struct yk_ray {
  float from[3];
  float dir[3];
  float tmin;
  float tmax; /* < 0 means unbounded, as scene_t::intersect (scene.cc:855-856) */
} yk_ray;

/* closest-hit record, 16 bytes: prim id (scene_t::update order) + t + b1,b2
 * (intersectData_t, surface.h:35-56); b0 = 1 - b1 - b2. prim = -1 on miss. */
typedef struct yk_hit {
  int32_t prim;
  float t;
  float b1;
  float b2;
} yk_hit;

typedef struct yk_scene_info {
  int32_t ntris, nmeshes, nmaterials, nlights;
  int32_t nnodes, nleaf_prims, max_depth;
  int32_t inodes, leaves, empty_leaves, leaf_refs, depth_limit_leaves, bad_split_leaves;
  float bound[6];
  double build_seconds;
  int32_t mode; /* YK_MODE_* of the built scene */
} yk_scene_info;

typedef struct yk_stats {
  uint64_t closest_rays;   /* scene_t::intersect calls (camera + bounces)          */
  uint64_t shadow_rays;    /* scene_t::isShadowed calls                            */
  uint64_t closest_nodes;  /* kd nodes visited by closest-hit traversal            */
  uint64_t closest_tris;   /* triangle tests (= leaf refs read) by closest-hit     */
  uint64_t shadow_nodes;
  uint64_t shadow_tris;
  uint64_t camera_samples;
  double ms_total;         /* wall time of the render passes (device-synchronised) */
  double ms_closest;       /* summed kernel time of the closest-hit kernels        */
  double ms_shadow;        /* summed kernel time of the any-hit kernels            */
  uint64_t closest_launches, shadow_launches;
  double ms_reduce;        /* yk_render_multi: wall time of the film reduces (peer
                              copies + sum), included in the call's time          */
} yk_stats;

typedef struct yk_scene yk_scene;   /* host scene + kd-tree (no GPU needed) */
typedef struct yk_device yk_device; /* one GPU with an uploaded scene       */

const char* yk_last_error(void);
const char* yk_version(void);

/* ---- host scene (scene_t geometry state machine + update) ---- */
int yk_scene_create(yk_scene** out);
void yk_scene_destroy(yk_scene* s);
int yk_scene_add_material(yk_scene* s, const yk_material* m, int32_t* id_out);
/* one TRIM mesh: points xyz (npoints*3), faces abc (nfaces*3); startTriMesh +
 * addVertex* + addTriangle* + endTriMesh (scene.cc:265-320,520-625) */
int yk_scene_add_mesh(yk_scene* s, const float* points, int32_t npoints, const int32_t* faces,
                      int32_t nfaces, int32_t material, int32_t* obj_id_out);
/* Vertex normals of mesh obj_id (triangle_t::na/nb/nc + triangleObject_t::normals):
 * normals xyz (nnormals*3), face_normals 3 indices per face (-1 = none),
 * flags YK_MESH_SMOOTH (triangleObject_t::is_smooth, set by smoothMesh or
 * exported normals, scene.cc:365-381) and YK_MESH_NORMALS_EXPORTED. */
enum { YK_MESH_SMOOTH = 1, YK_MESH_NORMALS_EXPORTED = 2 };
int yk_scene_set_mesh_normals(yk_scene* s, int32_t obj_id, const float* normals, int32_t nnormals,
                              const int32_t* face_normals, int32_t flags);
/* scene_t::startCurveMesh/addVertex/endCurveMesh (scene.cc:110-264): a hair
 * strand through npoints points, extruded to a triangular prism of
 * 6*(npoints-1)+2 triangles with the reference's radius law
 * (strand_start/end/shape) and vertex arithmetic. */
int yk_scene_add_curve(yk_scene* s, const float* points, int32_t npoints, int32_t material, float strand_start,
                       float strand_end, float strand_shape, int32_t* obj_id_out);
/* Scene mode (scene_t::setMode, xmlparser.cc:282-283; scene_t's default is
 * universal). YK_MODE_TRIANGLE: the tree holds the TRIM meshes and instances
 * (triKdTree_t); YK_MODE_UNIVERSAL: it holds the VTRIM meshes
 * (kdTree_t<primitive_t> over vTriangle_t, scene.cc:791-819), every one
 * whatever its visibility, whose any-hit test accepts t > tmin of the shifted
 * shadow ray (ray_kdtree.cc:936) and whose smooth shading weighs the first
 * vertex normal by intersectData_t::b0 = 0 (vTriangle_t::intersect never sets
 * it, triangle.cc:365-410) with normal index 0 meaning "none". */
enum { YK_MODE_TRIANGLE = 0, YK_MODE_UNIVERSAL = 1 };
int yk_scene_set_mode(yk_scene* s, int32_t mode);
/* the mesh type startTriMesh was given (object3d.h: TRIM 0, VTRIM 1) */
enum { YK_MESH_TRIM = 0, YK_MESH_VTRIM = 1 };
int yk_scene_set_mesh_type(yk_scene* s, int32_t obj_id, int32_t type);
/* mark a mesh as an instancing base: not traced itself (objData_t BASEMESH,
 * scene_t::update skips isBaseObject(), scene.cc:764) */
int yk_scene_set_mesh_base(yk_scene* s, int32_t obj_id);
/* scene_t::addInstance (scene.cc:983-1008): a triangleObjectInstance_t of a
 * base mesh with objToWorld as 16 floats, row-major (matrix4x4_t). Its prims
 * are flattened with the reference's vertex / normal transform arithmetic. */
int yk_scene_add_instance(yk_scene* s, int32_t base_obj_id, const float* obj_to_world, int32_t* obj_id_out);
int yk_scene_add_light(yk_scene* s, const yk_light* l);
int yk_scene_set_camera(yk_scene* s, const yk_camera* c);
/* scene_t::update: gather prims and build the kd-tree (scene.cc:748-785) */
int yk_scene_build(yk_scene* s);
int yk_scene_info_get(const yk_scene* s, yk_scene_info* out);
/* copy out flattened prims / tree; any pointer may be NULL */
int yk_scene_export(const yk_scene* s, float* tri_verts, int32_t* tri_material, float* tri_normal,
                    uint32_t* nodes, uint32_t* leaf_prims);
/* per-prim shading data: smooth flag (1 byte per prim) and the three vertex
 * normals getSurface interpolates (9 floats per prim, zero where not smooth) */
int yk_scene_export_shading(const yk_scene* s, uint8_t* smooth, float* vertex_normals);
int yk_scene_get_material(const yk_scene* s, int32_t i, yk_material* out);
int yk_scene_get_light(const yk_scene* s, int32_t i, yk_light* out);
int yk_scene_get_camera(const yk_scene* s, yk_camera* out);
/* procedural probe scenes: "cornell" (36 tris) or "bumpy" (2*nu*(nv-1)+2 tris);
 * fills the scene and the matching render params of BASELINE.md */
int yk_scene_generate(yk_scene* s, const char* name, int32_t p0, int32_t p1, int32_t resx,
                      int32_t resy, yk_render_params* params_out);
void yk_render_params_default(yk_render_params* p);
/* imageSpliter_t's "random" tile order (imagesplitter.cc:48): the row-major
 * list 0..ntiles-1 shuffled by libstdc++'s std::random_shuffle, whose
 * rand() is glibc's after srand(seed) -- seed 1 is a process that has not
 * called srand() or rand() before the film is set up. Uses a private
 * generator state (the caller's rand() is untouched). */
int yk_tile_order_random(int32_t ntiles, uint32_t seed, int32_t* order_out);
/* A live imageFilm_t -> render parameters: identifies the film's filter by
 * comparing its 16x16 filterTable (imagefilm.cc:119-165) with the box /
 * Mitchell / Gauss / Lanczos2 tables libyk builds, bit for bit, and takes its
 * filterw as is (p->filter, p->filter_width). YK_ERR_UNSUPPORTED when the
 * table is none of them or filterw lies outside [0.501, 4]. */
int yk_film_filter_from_table(const float* filter_table, float filterw, yk_render_params* p);

/* ---- reference object state ----
 * What the reference's constructors computed, for a plugin that reads it out
 * of the live objects: re-deriving it from the XML
 * parameters would not round-trip in float. The parameter-level calls above
 * convert to these states with the reference's constructor arithmetic. */
typedef struct yk_material_state {
  int32_t type;             /* YK_MAT_*                                                  */
  uint32_t bsdf_flags;      /* material_t::bsdfFlags (material.h:49-66)                 */
  float color[3];           /* shinyDiffuseMat_t::mDiffuseColor | lightMat_t::lightCol  */
  float diffuse_strength;   /* shinyDiffuseMat_t::mDiffuseStrength                      */
  float emit_color[3];      /* shinyDiffuseMat_t::mEmitColor (= emit strength * color)  */
  int32_t double_sided;     /* lightMat_t::doubleSided                                  */
  /* shinyDiffuseMat_t after config() (shinydiffuse.cc:27-80) */
  float mirror_color[3];    /* mMirrorColor                                              */
  float component[4];       /* getComponents: mirror, transparency, translucency,
                               diffuse strength; 0 where config() left it off           */
  int32_t ncomp;            /* nBSDF                                                     */
  uint32_t comp_flags[4];   /* cFlags                                                    */
  int32_t comp_index[4];    /* cIndex                                                    */
  float transmit_filter;    /* mTransmitFilterStrength                                   */
  int32_t has_fresnel;      /* mHasFresnelEffect                                         */
  float ior_squared;        /* mIOR_Squared                                              */
  int32_t oren_nayar;       /* mUseOrenNayar                                             */
  float oren_nayar_a;       /* mOrenNayar_A = 1 - 0.5 s^2/(s^2 + 0.33), in double        */
  float oren_nayar_b;       /* mOrenNayar_B = 0.45 s^2/(s^2 + 0.09), in double           */
} yk_material_state;

typedef struct yk_area_light_state { /* areaLight_t members (arealight.h:45-53) */
  float corner[3], to_x[3], to_y[3];
  float color[3];           /* includes pi * power (arealight.cc:38)                    */
  int32_t samples;
} yk_area_light_state;

typedef struct yk_dirac_light_state { /* pointLight_t / directionalLight_t members after their ctors */
  int32_t type;          /* YK_LIGHT_POINT or YK_LIGHT_DIRECTIONAL                                  */
  float position[3];     /* pointLight_t::position / directionalLight_t::position                  */
  float direction[3];    /* directional: normalized (directional.cc:53)                             */
  float color[3];        /* color * power (pointlight.cc:55, directional.cc:51)                     */
  float radius;          /* directional, non-infinite                                              */
  int32_t infinite;
} yk_dirac_light_state;

typedef struct yk_camera_state { /* perspectiveCam_t after setAxis (perspectiveCamera.cc:57-71) */
  float position[3], vright[3], vup[3], vto[3], cam_z[3];
  float near_p[3], far_p[3]; /* near_plane.p / far_plane.p (camera.h:54-57)            */
  int32_t resx, resy;
  /* depth of field (perspectiveCam_t ctor + setAxis): aperture (0 = pinhole),
   * dof_distance, dof_rt = aperture * camX, dof_up = aperture * camY, bokeh
   * type / bias and the polygon corner table LS (cos, sin pairs, up to 16) */
  float aperture, dof_distance;
  float dof_rt[3], dof_up[3];
  int32_t bokeh_type, bokeh_bias;
  float lens_ls[16];
} yk_camera_state;

int yk_scene_add_material_state(yk_scene* s, const yk_material_state* m, int32_t* id_out);
int yk_scene_add_area_light_state(yk_scene* s, const yk_area_light_state* l);
/* point / directional light (light_t::diracLight() == true): one shadow ray
 * per estimate, mcintegrator.cc:85-100 */
int yk_scene_add_dirac_light_state(yk_scene* s, const yk_dirac_light_state* l);
int yk_scene_get_dirac_light_state(const yk_scene* s, int32_t i, yk_dirac_light_state* out);
/* constBackground_t (textureback.cc:187-218, "constant", ibl off): camera
 * rays that miss add color*power. rgb NULL removes the background. */
int yk_scene_set_background(yk_scene* s, const float* rgb, float power);
/* has_out = 0 when the scene has no background */
int yk_scene_get_background(const yk_scene* s, float* rgb_out, int32_t* has_out);
int yk_scene_set_camera_state(yk_scene* s, const yk_camera_state* c);
int yk_scene_get_material_state(const yk_scene* s, int32_t i, yk_material_state* out);
int yk_scene_get_area_light_state(const yk_scene* s, int32_t i, yk_area_light_state* out);
int yk_scene_get_camera_state(const yk_scene* s, yk_camera_state* out);

/* ---- device ---- */
/* number of GPUs libyk can open (ordinals 0 .. n-1) */
int yk_device_count(int32_t* n);
int yk_device_open(int32_t ordinal, yk_device** out);
void yk_device_close(yk_device* d);
/* Uploads scene s (geometry, kd-tree, materials, lights, camera) and builds
 * the traversal's copies (node packets, leaf-ordered triangle records).
 * YK_ERR_ARG if the kd-tree has a leaf with 2^17 or more references (the
 * cooperative leaf test's limit) or 2^30 - 1 nodes or more (stack entries). */
int yk_device_upload(yk_device* d, const yk_scene* s);
int yk_device_sync(yk_device* d);
/* Abort polling (scene_t::getSignals() & Y_SIG_ABORT, integrator.cc:255):
 * renders on d call fn(user) between batches (tens of ms apart) and stop when
 * it returns non-zero -- the batches already running finish, the film holds
 * them, and the render returns YK_ERR_ABORTED. fn NULL removes the callback. */
typedef int32_t (*yk_abort_fn)(void* user);
int yk_device_set_abort(yk_device* d, yk_abort_fn fn, void* user);
/* hipStream_t the kernels run on, as an opaque pointer (for external timing) */
void* yk_device_stream(yk_device* d);

/* batched ray queries on device memory; bit-exact with the reference
 * triKdTree_t::Intersect (closest) and scene_t::isShadowed (any hit).
 * Closest: hits with tmin <= t < (tmax < 0 ? inf : tmax); prim -1 = miss.
 * Shadow: isShadowed(from, dir, tmin, tmax) semantics -- the query ray
 * starts at from + tmin*dir and reaches tmax - 2*tmin (scene.cc:884-889). */
int yk_trace_closest(yk_device* d, const yk_ray* d_rays, int64_t n, yk_hit* d_hits, yk_stats* st);
int yk_trace_shadow(yk_device* d, const yk_ray* d_rays, int64_t n, uint8_t* d_occluded, yk_stats* st);
/* scene_t::isShadowed(state, ray, maxDepth, filt) (scene.cc:904-928) ->
 * triKdTree_t::IntersectTS (kdtree.cc:953-1108): transparent materials let the
 * ray through and multiply d_filter (3 floats per ray) by getTransparency;
 * an opaque hit, or more than max_depth (<= 8) transparent ones, occludes. */
int yk_trace_shadow_filtered(yk_device* d, const yk_ray* d_rays, int64_t n, uint8_t* d_occluded, float* d_filter,
                             int32_t max_depth, yk_stats* st);

/* Render the tiles t with (t % nshards == shard) and accumulate the film
 * sums (R,G,B,A,weight per pixel, width*height*5 floats, pixel-major) into
 * d_film (device pointer, caller-allocated, caller-zeroed). */
int yk_render_shard(yk_device* d, const yk_render_params* p, int32_t shard, int32_t nshards,
                    float* d_film, yk_stats* st);
/* imageFilm_t::flush normalisation (+clampRGB0): film sums -> RGBA floats */
int yk_film_resolve(yk_device* d, const yk_render_params* p, const float* d_film, float* d_rgba);
/* convenience for host callers (the reference plugin): render the tiles of
 * `shard` and return the film sums (width*height*5 floats) in host memory */
int yk_render_film(yk_device* d, const yk_render_params* p, int32_t shard, int32_t nshards, float* film_host,
                   yk_stats* st);
/* Whole frame on ndev devices, replacing tiledIntegrator_t::render's worker
 * threads (integrator.cc:177-211): devs[i] renders the tiles t % ndev == i on
 * its own host thread, and the film sums are reduced on devs[0] by peer
 * copies over xGMI, in shard order, into film_host (width*height*5 floats).
 * With AA_passes > 1 the reduced film gives every pass's imageFilm_t::nextPass
 * flags (imagefilm.cc:213-289), so adaptive passes work across devices (per
 * pixel the result equals the 1-device film up to float summation order).
 * Every device must hold the same uploaded scene (YK_ERR_STATE otherwise) and,
 * for photon mapping / photon caustics, maps built with p->photon; a device
 * handle may appear only once, but two handles may be opened on one GPU.
 * The peer copies run concurrently (one stream per source GPU) and one pass
 * sums the films in shard order; the films and staging buffers stay on the
 * handles, so repeated calls allocate nothing. st->ms_reduce gets the reduce
 * time. Handles opened on one GPU share its constant memory (materials,
 * lights, camera): a handle re-binds it from its own upload before it
 * renders, so handles on one GPU that hold different scenes must not render
 * at the same time. "Same uploaded scene" means the same built scene and the
 * same camera, lights and materials at upload time (a camera changed between
 * two handles' uploads is refused). At most 16 handles (YK_ERR_UNSUPPORTED).
 * Memory: devs[0] keeps one staging film per peer-GPU shard and the sum film
 * (width*height*5 floats each) until yk_device_close. */
int yk_render_multi(yk_device* const* devs, int32_t ndev, const yk_render_params* p, float* film_host,
                    yk_stats* st);
/* convenience: whole frame on one device, RGBA float image to host memory */
int yk_render(yk_device* d, const yk_render_params* p, float* rgba_host, yk_stats* st);

/* ---- photon mapping (photonIntegrator_t, photonintegr.cc) ---- */
typedef struct yk_photon_info {
  int32_t diffuse_photons;   /* diffuseMap.nPhotons()                                */
  int32_t diffuse_paths;     /* diffuseMap.nPaths(): last path index that stored one */
  int32_t caustic_photons;   /* causticMap.nPhotons()                                */
  int32_t caustic_paths;
  int32_t rad_candidates;    /* radiance points chosen by ourRandom() < 0.125        */
  int32_t radiance_photons;  /* radiance points left after the 0.01*r elimination    */
  int32_t seed_out;          /* myseed after preprocess                              */
  int32_t tree_depth;        /* deepest diffuse-map kd-tree leaf                     */
  uint64_t photon_rays;      /* scene_t::intersect calls of the photon paths         */
  double ms_shoot, ms_tree, ms_pregather, ms_total;
} yk_photon_info;

/* photonIntegrator_t::preprocess (photonintegr.cc:126-633): shoot the diffuse
 * and caustic photons on the device, build the photon kd-trees
 * (kdtree::pointKdTree, pkdtree.h) on the host, pre-gather the radiance
 * photons of final gathering on the device. The maps stay resident for
 * yk_render_shard with p->integrator == YK_INTEGRATOR_PHOTON.
 * With p->integrator == YK_INTEGRATOR_PATH it is pathIntegrator_t::preprocess
 * for caustic_type photon / both (pathtracer.cc:76-129): only the caustic map
 * of mcIntegrator_t::createCausticMap (mcintegrator.cc:197-377). */
int yk_photon_build(yk_device* d, const yk_render_params* p, yk_photon_info* info);
enum { YK_PHOTON_MAP_DIFFUSE = 0, YK_PHOTON_MAP_CAUSTIC = 1, YK_PHOTON_MAP_RADIANCE = 2 };
/* copy a map out in photon-vector order: 9 floats per photon (pos, dir, color);
 * cap = capacity in photons; *n_out = photons in the map */
int yk_photon_export(yk_device* d, int32_t which, float* out, int32_t cap, int32_t* n_out);

/* ---- GPU kd-tree build ----
 * Replaces triKdTree_t's CPU constructor (kdtree.cc:75-666, called from
 * scene_t::update, scene.cc:782) for a device that already holds scene s
 * (yk_device_upload): a binned-SAH kd-tree built level by level on the device,
 * in the same node encoding, replacing the uploaded reference tree until the
 * next upload. Opt-in, with a documented tie-break: hits equal those of the
 * reference tree except for which primitive wins at exactly equal t
 * (DESIGN.md §4 "GPU kd-tree build"). flags must be 0. */
typedef struct yk_tree_info {
  int32_t nodes, interior, leaves, empty_leaves, max_depth;
  int64_t leaf_refs;
  double ms_build; /* host wall time of the call, uploads included */
} yk_tree_info;
int yk_device_build_tree(yk_device* d, const yk_scene* s, int32_t flags, yk_tree_info* info);
/* Copies the device's resident kd-tree (the uploaded reference tree, or the
 * one yk_device_build_tree made) to host memory in the export encoding of
 * yk_scene_export: 2 u32 per node (split bits / prim / leaf offset; axis |
 * right child or count << 2), leaf lists as u32 prim ids. With nodes / leaf
 * NULL only the counts are returned. Test and tooling hook: it lets checks
 * aim rays at the split planes of the tree actually traversed. */
int yk_device_export_tree(yk_device* d, uint32_t* nodes, int64_t node_cap, uint32_t* leaf, int64_t leaf_cap,
                          int64_t* nnodes_out, int64_t* nleaf_out);
/* Test-only hooks (the watchdog's tree damage) are declared in
 * yk_test_hooks.h, not here, and are disabled unless YK_DEBUG_HOOKS=1. */

#ifdef __cplusplus
}
#endif
#endif /* YK_API_H */
