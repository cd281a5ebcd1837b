// Reference-side integrator plugin: the drop-in that routes the reference's
// "pathtracing" / "directlighting" integrators to libyk (include/yk_api.h).
//
// This file is compiled INSIDE the reference's build tree, as one more plugin
// target next to src/integrators (it needs the reference's generated
// yafray_config.h, so it is not built in this repository). It talks to the GPU
// only through the C ABI, so the HIP library never sees a reference header or
// a C++ object.
//
// Flow (scene_t::render, scene.cc:905-950):
//   update() -> preprocess() -> render(film) -> cleanup() -> film->flush()
//   preprocess(): hand prims (scene_t::update order, scene.cc:760-781),
//                 material / area-light / camera *object state* to libyk,
//                 build the kd-tree, upload to the device
//   render():     yk_render_multi over all GPUs of the node (tiles t % N on
//                 GPU i, one host thread per GPU, film reduced over xGMI),
//                 then write the film sums into imageFilm_t's pixel buffer;
//                 the reference's own flush() normalises them exactly as
//                 k_film_resolve does
// What the GPU path cannot reproduce is refused with an error, never rendered
// differently: textured (shader-node) materials, other lights / backgrounds /
// cameras / volume integrators, film filters libyk does not build, premultiplied
// alpha (compounded per pixel, imagefilm.cc:502), depth passes.
#include <core_api/environment.h>
#include <core_api/imagefilm.h>
#include <core_api/scene.h>
#include <core_api/tiledintegrator.h>
#include <cameras/perspectiveCamera.h>
#include <lights/arealight.h>
#include <materials/shinydiff.h>
#include <yafraycore/meshtypes.h>
#include <yafraycore/triangle.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <typeinfo>
#include <vector>

#include "yk_api.h"

__BEGIN_YAFRAY

// ---- read protected/private members without editing the reference -------
// (explicit instantiation may name private members: [temp.explicit]/14)
template <class Tag>
struct member_of {
  static typename Tag::type ptr;
};
template <class Tag>
typename Tag::type member_of<Tag>::ptr;
template <class Tag, typename Tag::type P>
struct grant {
  grant() { member_of<Tag>::ptr = P; }
  static grant instance;
};
template <class Tag, typename Tag::type P>
grant<Tag, P> grant<Tag, P>::instance;

#define YK_COMMA ,
#define YK_MEMBER(name, cls, mtype, member)             \
  struct name {                                         \
    typedef mtype cls::*type;                           \
  };                                                    \
  template struct grant<name, &cls::member>;
YK_MEMBER(SceneMeshes, scene_t, std::map<objID_t YK_COMMA objData_t>, meshes)
YK_MEMBER(SceneObjects, scene_t, std::map<objID_t YK_COMMA object3d_t*>, objects)
YK_MEMBER(SceneMode, scene_t, int, mode)
YK_MEMBER(MObjTris, meshObject_t, std::vector<vTriangle_t>, triangles)
YK_MEMBER(MObjBsTris, meshObject_t, std::vector<bsTriangle_t>, s_triangles)
YK_MEMBER(MObjPoints, meshObject_t, std::vector<point3d_t>, points)
YK_MEMBER(MObjNormals, meshObject_t, std::vector<normal_t>, normals)
YK_MEMBER(MObjSmooth, meshObject_t, bool, is_smooth)
YK_MEMBER(VTriPa, vTriangle_t, int, pa)
YK_MEMBER(VTriPb, vTriangle_t, int, pb)
YK_MEMBER(VTriPc, vTriangle_t, int, pc)
YK_MEMBER(VTriNa, vTriangle_t, int, na)
YK_MEMBER(VTriNb, vTriangle_t, int, nb)
YK_MEMBER(VTriNc, vTriangle_t, int, nc)
YK_MEMBER(TriPa, triangle_t, int, pa)
YK_MEMBER(TriPb, triangle_t, int, pb)
YK_MEMBER(TriPc, triangle_t, int, pc)
YK_MEMBER(TriNa, triangle_t, int, na)
YK_MEMBER(TriNb, triangle_t, int, nb)
YK_MEMBER(TriNc, triangle_t, int, nc)
YK_MEMBER(MeshPoints, triangleObject_t, std::vector<point3d_t>, points)
YK_MEMBER(MeshNormals, triangleObject_t, std::vector<normal_t>, normals)
YK_MEMBER(MeshSmooth, triangleObject_t, bool, is_smooth)
YK_MEMBER(MeshNormalsExported, triangleObject_t, bool, normals_exported)
YK_MEMBER(InstToWorld, triangleObjectInstance_t, matrix4x4_t, objToWorld)
YK_MEMBER(InstBase, triangleObjectInstance_t, triangleObject_t*, mBase)
YK_MEMBER(SdColor, shinyDiffuseMat_t, color_t, mDiffuseColor)
YK_MEMBER(SdStrength, shinyDiffuseMat_t, float, mDiffuseStrength)
YK_MEMBER(SdEmit, shinyDiffuseMat_t, color_t, mEmitColor)
YK_MEMBER(SdMirrorColor, shinyDiffuseMat_t, color_t, mMirrorColor)
YK_MEMBER(SdMirror, shinyDiffuseMat_t, float, mMirrorStrength)
YK_MEMBER(SdTransp, shinyDiffuseMat_t, float, mTransparencyStrength)
YK_MEMBER(SdTransl, shinyDiffuseMat_t, float, mTranslucencyStrength)
YK_MEMBER(SdFilter, shinyDiffuseMat_t, float, mTransmitFilterStrength)
YK_MEMBER(SdIsMirror, shinyDiffuseMat_t, bool, mIsMirror)
YK_MEMBER(SdIsTransparent, shinyDiffuseMat_t, bool, mIsTransparent)
YK_MEMBER(SdIsTranslucent, shinyDiffuseMat_t, bool, mIsTranslucent)
YK_MEMBER(SdIsDiffuse, shinyDiffuseMat_t, bool, mIsDiffuse)
YK_MEMBER(SdFresnel, shinyDiffuseMat_t, bool, mHasFresnelEffect)
YK_MEMBER(SdIor2, shinyDiffuseMat_t, float, mIOR_Squared)
YK_MEMBER(SdOrenNayar, shinyDiffuseMat_t, bool, mUseOrenNayar)
YK_MEMBER(SdOrenNayarA, shinyDiffuseMat_t, float, mOrenNayar_A)
YK_MEMBER(SdOrenNayarB, shinyDiffuseMat_t, float, mOrenNayar_B)
YK_MEMBER(SdNBSDF, shinyDiffuseMat_t, int, nBSDF)
YK_MEMBER(SdCFlags, shinyDiffuseMat_t, BSDF_t[4], cFlags)
YK_MEMBER(SdCIndex, shinyDiffuseMat_t, int[4], cIndex)
YK_MEMBER(SdDiffuseShader, shinyDiffuseMat_t, shaderNode_t*, mDiffuseShader)
YK_MEMBER(SdBumpShader, shinyDiffuseMat_t, shaderNode_t*, mBumpShader)
YK_MEMBER(SdMirrorShader, shinyDiffuseMat_t, shaderNode_t*, mMirrorShader)
YK_MEMBER(SdMirrorColorShader, shinyDiffuseMat_t, shaderNode_t*, mMirrorColorShader)
YK_MEMBER(SdTranspShader, shinyDiffuseMat_t, shaderNode_t*, mTransparencyShader)
YK_MEMBER(SdTranslShader, shinyDiffuseMat_t, shaderNode_t*, mTranslucencyShader)
YK_MEMBER(AlCorner, areaLight_t, point3d_t, corner)
YK_MEMBER(AlToX, areaLight_t, vector3d_t, toX)
YK_MEMBER(AlToY, areaLight_t, vector3d_t, toY)
YK_MEMBER(AlColor, areaLight_t, color_t, color)
YK_MEMBER(AlSamples, areaLight_t, int, samples)
YK_MEMBER(CamPos, camera_t, point3d_t, position)
YK_MEMBER(CamZ, camera_t, vector3d_t, camZ)
YK_MEMBER(CamVto, camera_t, vector3d_t, vto)
YK_MEMBER(CamVup, camera_t, vector3d_t, vup)
YK_MEMBER(CamVright, camera_t, vector3d_t, vright)
YK_MEMBER(CamNear, camera_t, plane_t, near_plane)
YK_MEMBER(CamFar, camera_t, plane_t, far_plane)
YK_MEMBER(CamAperture, perspectiveCam_t, PFLOAT, aperture)
YK_MEMBER(CamDofDistance, perspectiveCam_t, PFLOAT, dof_distance)
YK_MEMBER(CamDofRt, perspectiveCam_t, vector3d_t, dof_rt)
YK_MEMBER(CamDofUp, perspectiveCam_t, vector3d_t, dof_up)
YK_MEMBER(CamBokeh, perspectiveCam_t, perspectiveCam_t::bokehType, bkhtype)
YK_MEMBER(CamBokehBias, perspectiveCam_t, perspectiveCam_t::bkhBiasType, bkhbias)
YK_MEMBER(CamLS, perspectiveCam_t, std::vector<PFLOAT>, LS)
YK_MEMBER(FilmImage, imageFilm_t, rgba2DImage_t*, image)
YK_MEMBER(FilmCx0, imageFilm_t, int, cx0)
YK_MEMBER(FilmCy0, imageFilm_t, int, cy0)
YK_MEMBER(FilmFilterW, imageFilm_t, float, filterw)
YK_MEMBER(FilmTable, imageFilm_t, float*, filterTable)
YK_MEMBER(FilmTileSize, imageFilm_t, int, tileSize)
YK_MEMBER(FilmPremult, imageFilm_t, bool, premultAlpha)
YK_MEMBER(FilmSplitter, imageFilm_t, imageSpliter_t*, splitter)
#define GET(obj, Tag) ((obj).*member_of<Tag>::ptr)

// pointLight_t, directionalLight_t and constBackground_t are defined inside
// their plugins' .cc files (pointlight.cc:27-45, directional.cc:27-50,
// textureback.cc:59-69), so no header declares them. These mirror their
// member layout (same compiler and ABI as the reference build, SURVEY.md
// §8(b)); the object is identified by its typeid name before the cast.
// The integrator never constructs them.
struct PointLightLayout : public light_t {
  point3d_t position;
  color_t color;
  float intensity;
};
struct DirectionalLightLayout : public light_t {
  point3d_t position;
  color_t color;
  vector3d_t direction, du, dv;
  float intensity;
  PFLOAT radius;
  float areaPdf;
  PFLOAT worldRadius;
  bool infinite;
  int majorAxis;
};
struct ConstBackgroundLayout : public background_t {
  color_t color;
};

static void put3(float* d, float x, float y, float z) { d[0] = x; d[1] = y; d[2] = z; }

class gpuTiledIntegrator_t : public tiledIntegrator_t {
 public:
  gpuTiledIntegrator_t(const yk_render_params& p, const char* name) : params(p) {
    type = SURFACE;
    integratorName = name;
    integratorShortName = name;
  }
  ~gpuTiledIntegrator_t() { release(); }

  bool preprocess() override {
    release();
    if (yk_scene_create(&ys) != YK_OK) return fail();
    // materials: object state of the materials the prims reference
    std::map<const material_t*, int32_t> mat_ids;
    std::map<objID_t, objData_t>& meshes = GET(*scene, SceneMeshes);
    // yk object ids of each reference mesh (one per material run), so that
    // instances (scene_t::addInstance, scene.cc:983-1008) can name their base
    std::map<const triangleObject_t*, std::vector<int32_t>> yk_ids;
    // universal mode (scene_t::mode 1): the tree holds the VTRIM meshes'
    // vTriangle_t prims, every one whatever its visibility (scene.cc:791-819)
    const bool universal = GET(*scene, SceneMode) != 0;
    if (universal) {
      if (yk_scene_set_mode(ys, YK_MODE_UNIVERSAL) != YK_OK) return fail();
      if (!GET(*scene, SceneObjects).empty()) return unsupported("non-mesh primitives are not on the GPU path");
      for (auto& kv : meshes) {
        objData_t& dat = kv.second;
        if (dat.type == TRIM) continue;  // not in the universal tree
        if (dat.type != VTRIM || !GET(*dat.mobj, MObjBsTris).empty())
          return unsupported("bezier (MTRIM) meshes are not on the GPU path");
        const std::vector<vTriangle_t>& tris = GET(*dat.mobj, MObjTris);
        // points keep their orco interleaved (pa + 1): faces index them as stored
        const std::vector<point3d_t>& pts = GET(*dat.mobj, MObjPoints);
        std::vector<float> xyz(3 * pts.size());
        for (size_t i = 0; i < pts.size(); ++i) put3(&xyz[3 * i], pts[i].x, pts[i].y, pts[i].z);
        const std::vector<normal_t>& nrm = GET(*dat.mobj, MObjNormals);
        std::vector<float> nxyz(3 * nrm.size());
        for (size_t i = 0; i < nrm.size(); ++i) put3(&nxyz[3 * i], nrm[i].x, nrm[i].y, nrm[i].z);
        for (size_t a = 0; a < tris.size();) {  // one yk mesh per run of prims with the same material
          const material_t* m = tris[a].getMaterial();
          size_t b = a;
          std::vector<int32_t> faces, fnrm;
          while (b < tris.size() && tris[b].getMaterial() == m) {
            faces.push_back(GET(tris[b], VTriPa));
            faces.push_back(GET(tris[b], VTriPb));
            faces.push_back(GET(tris[b], VTriPc));
            for (int k : {GET(tris[b], VTriNa), GET(tris[b], VTriNb), GET(tris[b], VTriNc)})
              fnrm.push_back(k >= 0 && k < (int)nrm.size() ? k : -1);
            ++b;
          }
          int32_t mid, oid;
          if (!material_id(m, mat_ids, mid)) return false;
          if (yk_scene_add_mesh(ys, xyz.data(), (int32_t)pts.size(), faces.data(), (int32_t)(faces.size() / 3), mid,
                                &oid) != YK_OK ||
              yk_scene_set_mesh_type(ys, oid, YK_MESH_VTRIM) != YK_OK)
            return fail();
          if (GET(*dat.mobj, MObjSmooth) &&
              yk_scene_set_mesh_normals(ys, oid, nxyz.data(), (int32_t)nrm.size(), fnrm.data(), YK_MESH_SMOOTH) != YK_OK)
            return fail();
          a = b;
        }
      }
    }
    for (auto& kv : meshes) {
      objData_t& dat = kv.second;
      if (universal || !dat.obj->isVisible() || dat.type != TRIM) continue;
      if (triangleObjectInstance_t* inst = dynamic_cast<triangleObjectInstance_t*>(dat.obj)) {
        // prims of an instance = the base's prims in order: instance each run
        const matrix4x4_t& M = GET(*inst, InstToWorld);
        float m16[16];
        for (int r = 0; r < 4; ++r)
          for (int c = 0; c < 4; ++c) m16[4 * r + c] = M[r][c];
        auto it = yk_ids.find(GET(*inst, InstBase));
        if (it == yk_ids.end()) return unsupported("instance of a mesh the GPU path did not load");
        for (int32_t base_id : it->second)
          if (yk_scene_add_instance(ys, base_id, m16, nullptr) != YK_OK) return fail();
        continue;
      }
      // base meshes are loaded too (marked base: not traced, scene.cc:765)
      const int n = dat.obj->numPrimitives();
      std::vector<const triangle_t*> prims(n);
      dat.obj->getPrimitives(prims.data());
      const std::vector<point3d_t>& pts = GET(*dat.obj, MeshPoints);
      std::vector<float> xyz(3 * pts.size());
      for (size_t i = 0; i < pts.size(); ++i) put3(&xyz[3 * i], pts[i].x, pts[i].y, pts[i].z);
      const std::vector<normal_t>& nrm = GET(*dat.obj, MeshNormals);
      std::vector<float> nxyz(3 * nrm.size());
      for (size_t i = 0; i < nrm.size(); ++i) put3(&nxyz[3 * i], nrm[i].x, nrm[i].y, nrm[i].z);
      const int32_t flags = (GET(*dat.obj, MeshSmooth) ? YK_MESH_SMOOTH : 0) |
                            (GET(*dat.obj, MeshNormalsExported) ? YK_MESH_NORMALS_EXPORTED : 0);
      std::vector<int32_t>& ids = yk_ids[dat.obj];
      // one yk mesh per run of prims with the same material, prim order kept
      for (int a = 0; a < n;) {
        const material_t* m = prims[a]->getMaterial();
        int b = a;
        std::vector<int32_t> faces, fnrm;
        while (b < n && prims[b]->getMaterial() == m) {
          faces.push_back(GET(*prims[b], TriPa));
          faces.push_back(GET(*prims[b], TriPb));
          faces.push_back(GET(*prims[b], TriPc));
          for (int k : {GET(*prims[b], TriNa), GET(*prims[b], TriNb), GET(*prims[b], TriNc)})
            fnrm.push_back(k >= 0 && k < (int)nrm.size() ? k : -1);
          ++b;
        }
        int32_t mid, oid;
        if (!material_id(m, mat_ids, mid)) return false;
        if (yk_scene_add_mesh(ys, xyz.data(), (int32_t)pts.size(), faces.data(), (int32_t)(faces.size() / 3),
                              mid, &oid) != YK_OK)
          return fail();
        if (flags && yk_scene_set_mesh_normals(ys, oid, nxyz.data(), (int32_t)nrm.size(), fnrm.data(), flags) != YK_OK)
          return fail();
        if (dat.obj->isBaseObject() && yk_scene_set_mesh_base(ys, oid) != YK_OK) return fail();
        ids.push_back(oid);
        a = b;
      }
    }
    for (light_t* l : scene->lights) {
      const std::string tn = typeid(*l).name();
      if (tn == "N7yafaray12pointLight_tE") {
        const PointLightLayout* pl = static_cast<const PointLightLayout*>(l);
        yk_dirac_light_state d{};
        d.type = YK_LIGHT_POINT;
        put3(d.position, pl->position.x, pl->position.y, pl->position.z);
        put3(d.color, pl->color.R, pl->color.G, pl->color.B);
        if (yk_scene_add_dirac_light_state(ys, &d) != YK_OK) return fail();
        continue;
      }
      if (tn == "N7yafaray18directionalLight_tE") {
        const DirectionalLightLayout* dl = static_cast<const DirectionalLightLayout*>(l);
        yk_dirac_light_state d{};
        d.type = YK_LIGHT_DIRECTIONAL;
        put3(d.position, dl->position.x, dl->position.y, dl->position.z);
        put3(d.direction, dl->direction.x, dl->direction.y, dl->direction.z);
        put3(d.color, dl->color.R, dl->color.G, dl->color.B);
        d.radius = dl->radius;
        d.infinite = dl->infinite ? 1 : 0;
        if (yk_scene_add_dirac_light_state(ys, &d) != YK_OK) return fail();
        continue;
      }
      areaLight_t* al = dynamic_cast<areaLight_t*>(l);
      if (!al) return unsupported("only area, point and directional lights run on the GPU path");
      yk_area_light_state s{};
      const point3d_t& c = GET(*al, AlCorner);
      const vector3d_t &x = GET(*al, AlToX), &y = GET(*al, AlToY);
      const color_t& col = GET(*al, AlColor);
      put3(s.corner, c.x, c.y, c.z);
      put3(s.to_x, x.x, x.y, x.z);
      put3(s.to_y, y.x, y.y, y.z);
      put3(s.color, col.R, col.G, col.B);
      s.samples = GET(*al, AlSamples);
      if (yk_scene_add_area_light_state(ys, &s) != YK_OK) return fail();
    }
    if (const background_t* bg = scene->getBackground()) {
      if (std::string(typeid(*bg).name()) != "N7yafaray17constBackground_tE")
        return unsupported("only the constant background runs on the GPU path");
      const color_t& c = static_cast<const ConstBackgroundLayout*>(bg)->color;
      const float rgb[3] = {c.R, c.G, c.B};
      if (yk_scene_set_background(ys, rgb, 1.0f) != YK_OK) return fail();  // color already * power
    }
    const perspectiveCam_t* cam = dynamic_cast<const perspectiveCam_t*>(scene->getCamera());
    if (!cam) return unsupported("only the perspective camera runs on the GPU path");
    yk_camera_state cs{};
    const camera_t& cb = *cam;
    const point3d_t& pos = GET(cb, CamPos);
    const vector3d_t &z = GET(cb, CamZ), &vto = GET(cb, CamVto), &vup = GET(cb, CamVup),
                     &vr = GET(cb, CamVright);
    put3(cs.position, pos.x, pos.y, pos.z);
    put3(cs.cam_z, z.x, z.y, z.z);
    put3(cs.vto, vto.x, vto.y, vto.z);
    put3(cs.vup, vup.x, vup.y, vup.z);
    put3(cs.vright, vr.x, vr.y, vr.z);
    const vector3d_t &np = GET(cb, CamNear).p, &fp = GET(cb, CamFar).p;
    put3(cs.near_p, np.x, np.y, np.z);
    put3(cs.far_p, fp.x, fp.y, fp.z);
    cs.resx = cam->resX();
    cs.resy = cam->resY();
    // depth of field: the lens state the constructor and setAxis computed
    // (perspectiveCamera.cc:29-71); libyk samples it as renderTile does
    const perspectiveCam_t& pc = *cam;
    cs.aperture = GET(pc, CamAperture);
    cs.dof_distance = GET(pc, CamDofDistance);
    const vector3d_t &drt = GET(pc, CamDofRt), &dup = GET(pc, CamDofUp);
    put3(cs.dof_rt, drt.x, drt.y, drt.z);
    put3(cs.dof_up, dup.x, dup.y, dup.z);
    cs.bokeh_type = (int32_t)GET(pc, CamBokeh);
    cs.bokeh_bias = (int32_t)GET(pc, CamBokehBias);
    const std::vector<PFLOAT>& ls = GET(pc, CamLS);
    if (ls.size() > 16) return unsupported("bokeh polygon table larger than 16 entries");
    for (size_t i = 0; i < ls.size(); ++i) cs.lens_ls[i] = ls[i];
    if (yk_scene_set_camera_state(ys, &cs) != YK_OK) return fail();
    // the empty volume integrator leaves integrate()'s colour as is
    // (pathtracer.cc:323-328 with transmittance 1, integrate 0)
    if (scene->volIntegrator && std::string(typeid(*scene->volIntegrator).name()) != "N7yafaray21EmptyVolumeIntegratorE")
      return unsupported("volume integrators other than \"none\" are not on the GPU path");
    if (yk_scene_build(ys) != YK_OK) return fail();
    // every GPU of the node holds the scene (replicated
    // scene, tiles sharded); "gpus" > 0 limits the count
    int32_t ndev = 0;
    if (yk_device_count(&ndev) != YK_OK || ndev < 1) return unsupported("no GPU for the GPU path");
    if (max_gpus > 0 && ndev > max_gpus) ndev = max_gpus;
    for (int32_t g = 0; g < ndev; ++g) {
      yk_device* d = nullptr;
      if (yk_device_open(g, &d) != YK_OK) return fail();
      devs.push_back(d);
      if (yk_device_upload(d, ys) != YK_OK) return fail();
      if (yk_device_set_abort(d, &gpuTiledIntegrator_t::abort_requested, scene) != YK_OK) return fail();
      if (gpu_tree) {  // opt-in: replace the reference tree by the device-built one
        yk_tree_info ti{};
        if (yk_device_build_tree(d, ys, 0, &ti) != YK_OK) return fail();
        if (g == 0)
          Y_INFO << integratorName << ": device kd-tree, " << ti.nodes << " nodes (" << ti.ms_build << " ms)" << yendl;
      }
    }
    const bool pt_photons = params.integrator == YK_INTEGRATOR_PATH &&
                            (params.caustic_type == YK_CAUSTIC_PHOTON || params.caustic_type == YK_CAUSTIC_BOTH);
    // photon maps: every GPU builds the same maps from the same inputs (the
    // build is deterministic), so each holds a replica
    if (pt_photons) {
      // pathIntegrator_t::preprocess -> mcIntegrator_t::createCausticMap
      // (pathtracer.cc:90-93, mcintegrator.cc:197-377) on the device; the
      // caustic pass draws no ourRandom() numbers
      yk_photon_info info{};
      for (yk_device* d : devs)
        if (yk_photon_build(d, &params, &info) != YK_OK) return fail();
      Y_INFO << integratorName << ": " << info.caustic_photons << " caustic photons (" << info.ms_total << " ms)"
             << yendl;
    }
    if (params.integrator == YK_INTEGRATOR_PHOTON) {
      // photonIntegrator_t::preprocess (photonintegr.cc:126-633) on the
      // device; the radiance points draw from the global ourRandom() state
      // (myseed, vector3d.cc:185), which continues afterwards as if the
      // reference had drawn them
      params.photon.seed = myseed;
      yk_photon_info info{};
      for (yk_device* d : devs)
        if (yk_photon_build(d, &params, &info) != YK_OK) return fail();
      myseed = info.seed_out;
      Y_INFO << integratorName << ": " << info.diffuse_photons << " diffuse photons, " << info.radiance_photons
             << " radiance photons (" << info.ms_total << " ms)" << yendl;
    }
    Y_INFO << integratorName << ": rendering on " << devs.size() << " GPU(s)" << yendl;
    return true;
  }

  bool render(imageFilm_t* film) override {
    // render area and AA settings as the film / scene hold them
    int aa_inc;
    CFLOAT thr;
    scene->getAAParameters(params.aa_samples, params.aa_passes, aa_inc, thr);
    // AA_passes > 1: libyk runs nextPass's adaptive passes itself, with the
    // flags of the film reduced over all GPUs
    params.aa_inc_samples = aa_inc;
    params.aa_threshold = (float)thr;
    rgba2DImage_t* img = GET(*film, FilmImage);
    const int w = img->getWidth(), h = img->getHeight();
    params.width = w;
    params.height = h;
    params.xstart = GET(*film, FilmCx0);
    params.ystart = GET(*film, FilmCy0);
    params.tile_size = GET(*film, FilmTileSize);
    // filter: libyk names it from the table the film built (imagefilm.cc:
    // 119-165) and takes filterw as the film holds it; a table it does not
    // build is refused
    if (yk_film_filter_from_table(GET(*film, FilmTable), GET(*film, FilmFilterW), &params) != YK_OK) return fail();
    if (GET(*film, FilmPremult)) return unsupported("premultiplied alpha films are not on the GPU path");
    if (scene->doDepth()) return unsupported("depth passes are not on the GPU path");
    // as tiledIntegrator_t::render does (integrator.cc:148): clear the film and
    // build its tile splitter, whose order ("tiles_order": row-major, or
    // std::random_shuffle for "random", imagesplitter.cc:29-53) is the order
    // imageFilm_t::nextArea hands the tiles out and so the splat order
    film->init(params.aa_passes);
    std::vector<int32_t> order;
    if (imageSpliter_t* sp = GET(*film, FilmSplitter)) {
      const int ts = params.tile_size, ntx = (w + ts - 1) / ts;
      renderArea_t a;
      for (int n = 0; sp->getArea(n, a); ++n)
        order.push_back((int32_t)(((a.Y - params.ystart) / ts) * ntx + (a.X - params.xstart) / ts));
    }
    params.tile_order = order.empty() ? nullptr : order.data();
    params.tile_order_len = (int32_t)order.size();
    std::vector<float> sums((size_t)w * h * 5);
    const int rc = yk_render_multi(devs.data(), (int32_t)devs.size(), &params, sums.data(), nullptr);
    params.tile_order = nullptr;  // `order` ends with this call
    params.tile_order_len = 0;
    if (rc != YK_OK && rc != YK_ERR_ABORTED) return fail();  // aborted: keep what was rendered, as renderTile does
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) {
        const float* s = &sums[5 * ((size_t)j * w + i)];
        pixel_t& px = (*img)(i, j);
        px.col = colorA_t(s[0], s[1], s[2], s[3]);
        px.weight = s[4];
      }
    return true;
  }

  void cleanup() override { release(); }

  // unused: render() never calls renderTile()
  colorA_t integrate(renderState_t&, diffRay_t&) const override { return colorA_t(0.f); }

  // Y_SIG_ABORT polling (renderTile, integrator.cc:255), called by libyk
  // between batches on every GPU's host thread
  static int32_t abort_requested(void* user) {
    return (static_cast<const scene_t*>(user)->getSignals() & Y_SIG_ABORT) ? 1 : 0;
  }

  static integrator_t* factory_path(paraMap_t& pm, renderEnvironment_t&) {
    yk_render_params p;
    yk_render_params_default(&p);  // pathIntegrator_t::factory defaults
    p.integrator = YK_INTEGRATOR_PATH;
    pm.getParam("raydepth", p.raydepth);
    pm.getParam("path_samples", p.path_samples);
    pm.getParam("bounces", p.bounces);
    read_shadow_params(pm, p);  // pathtracer.cc:337-353
    bool bg = true;
    pm.getParam("bg_transp", bg);
    p.transp_background = bg;
    bool use_sss = false;
    pm.getParam("useSSS", use_sss);
    if (use_sss) { Y_ERROR << "PathTracer: SSS photons are not on the GPU path" << yendl; return nullptr; }
    const std::string* cm = nullptr;
    // pathIntegrator_t::factory (pathtracer.cc:367-385): "photon" / "both"
    // read the caustic-map parameters with the factory's defaults
    if (pm.getParam("caustic_type", cm)) {
      bool use_photons = false;
      if (*cm == "photon") { p.caustic_type = YK_CAUSTIC_PHOTON; use_photons = true; }
      else if (*cm == "both") { p.caustic_type = YK_CAUSTIC_BOTH; use_photons = true; }
      else if (*cm == "none") p.caustic_type = YK_CAUSTIC_NONE;
      if (use_photons) {
        double c_rad = 0.25;
        int c_depth = 10, search = 100, photons = 500000;
        pm.getParam("photons", photons);
        pm.getParam("caustic_mix", search);
        pm.getParam("caustic_depth", c_depth);
        pm.getParam("caustic_radius", c_rad);
        p.photon.caustic_photons = photons;
        p.photon.caustic_mix = search;
        p.photon.bounces = c_depth;
        p.photon.caustic_radius = (float)c_rad;
      }
    }
    auto* it = new gpuTiledIntegrator_t(p, "PathTracer");
    it->read_plugin_params(pm);
    return it;
  }
  static integrator_t* factory_direct(paraMap_t& pm, renderEnvironment_t&) {
    yk_render_params p;
    yk_render_params_default(&p);
    p.integrator = YK_INTEGRATOR_DIRECT;
    pm.getParam("raydepth", p.raydepth);
    read_shadow_params(pm, p);  // directlight.cc factory
    bool bg = true;
    pm.getParam("bg_transp", bg);
    p.transp_background = bg;
    auto* it = new gpuTiledIntegrator_t(p, "DirectLight");
    it->read_plugin_params(pm);
    return it;
  }
  // "transpShad" / "shadowDepth" -> mcIntegrator_t::trShad / sDepth; the
  // device keeps at most 8 filtered surfaces per shadow ray
  static void read_shadow_params(paraMap_t& pm, yk_render_params& p) {
    bool ts = false;
    pm.getParam("transpShad", ts);
    p.transp_shadows = ts;
    pm.getParam("shadowDepth", p.shadow_depth);
  }
  // photonIntegrator_t::factory (photonintegr.cc:884-960): same parameter
  // names and defaults (yk_render_params_default)
  static integrator_t* factory_photon(paraMap_t& pm, renderEnvironment_t&) {
    yk_render_params p;
    yk_render_params_default(&p);
    p.integrator = YK_INTEGRATOR_PHOTON;
    yk_photon_params& q = p.photon;
    bool transp_shad = false, fg = true, show_map = false, bg = true;
    int raydepth = 5, photons = q.photons, cphotons = q.caustic_photons, search = q.search, bounces = q.bounces,
        fg_samples = q.fg_samples, fg_bounces = q.fg_bounces;
    float ds_rad = q.diffuse_radius, c_rad = q.caustic_radius;
    pm.getParam("transpShad", transp_shad);
    pm.getParam("raydepth", raydepth);
    pm.getParam("photons", photons);
    pm.getParam("cPhotons", cphotons);
    pm.getParam("diffuseRadius", ds_rad);
    pm.getParam("causticRadius", c_rad);
    pm.getParam("search", search);
    int caustic_mix = search;
    pm.getParam("caustic_mix", caustic_mix);
    pm.getParam("bounces", bounces);
    pm.getParam("finalGather", fg);
    pm.getParam("fg_samples", fg_samples);
    pm.getParam("fg_bounces", fg_bounces);
    float gather_dist = ds_rad;
    pm.getParam("fg_min_pathlen", gather_dist);
    pm.getParam("show_map", show_map);
    pm.getParam("bg_transp", bg);
    bool use_sss = false;
    pm.getParam("useSSS", use_sss);
    p.transp_shadows = transp_shad;
    pm.getParam("shadowDepth", p.shadow_depth);
    if (use_sss) { Y_ERROR << "PhotonMap: SSS photons are not on the GPU path" << yendl; return nullptr; }
    p.raydepth = raydepth;
    p.transp_background = bg;
    q.photons = photons;
    q.caustic_photons = cphotons;
    q.diffuse_radius = ds_rad;
    q.caustic_radius = c_rad;
    q.search = search;
    q.caustic_mix = caustic_mix;
    q.bounces = bounces;
    q.final_gather = fg;
    q.fg_samples = fg_samples;
    q.fg_bounces = fg_bounces;
    q.fg_min_pathlen = gather_dist;
    q.show_map = show_map;
    auto* it = new gpuTiledIntegrator_t(p, "PhotonMap");
    it->read_plugin_params(pm);
    return it;
  }

 private:
  // GPU-path options: "gpu_kdtree" (device-built tree, documented tie-break)
  // and "gpus" (> 0: at most this many GPUs)
  void read_plugin_params(paraMap_t& pm) {
    pm.getParam("gpu_kdtree", gpu_tree);
    pm.getParam("gpus", max_gpus);
  }
  bool material_id(const material_t* m, std::map<const material_t*, int32_t>& ids, int32_t& id) {
    auto it = ids.find(m);
    if (it != ids.end()) return (id = it->second), true;
    yk_material_state s{};
    s.bsdf_flags = m->getFlags();
    if (const shinyDiffuseMat_t* sd = dynamic_cast<const shinyDiffuseMat_t*>(m)) {
      s.type = YK_MAT_SHINYDIFFUSE;
      if (GET(*sd, SdDiffuseShader) || GET(*sd, SdBumpShader) || GET(*sd, SdMirrorShader) ||
          GET(*sd, SdMirrorColorShader) || GET(*sd, SdTranspShader) || GET(*sd, SdTranslShader))
        return unsupported("textured (shader-node) shinydiffuse is not on the GPU path");
      const color_t &c = GET(*sd, SdColor), &e = GET(*sd, SdEmit), &mc = GET(*sd, SdMirrorColor);
      put3(s.color, c.R, c.G, c.B);
      put3(s.emit_color, e.R, e.G, e.B);
      put3(s.mirror_color, mc.R, mc.G, mc.B);
      s.diffuse_strength = GET(*sd, SdStrength);
      // getComponents (shinydiffuse.cc:82-98): the strengths of the
      // components config() enabled, 0 elsewhere
      s.component[0] = GET(*sd, SdIsMirror) ? GET(*sd, SdMirror) : 0.f;
      s.component[1] = GET(*sd, SdIsTransparent) ? GET(*sd, SdTransp) : 0.f;
      s.component[2] = GET(*sd, SdIsTranslucent) ? GET(*sd, SdTransl) : 0.f;
      s.component[3] = GET(*sd, SdIsDiffuse) ? GET(*sd, SdStrength) : 0.f;
      s.ncomp = GET(*sd, SdNBSDF);
      for (int k = 0; k < 4; ++k) {
        s.comp_flags[k] = GET(*sd, SdCFlags)[k];
        s.comp_index[k] = GET(*sd, SdCIndex)[k];
      }
      s.transmit_filter = GET(*sd, SdFilter);
      s.has_fresnel = GET(*sd, SdFresnel) ? 1 : 0;
      s.ior_squared = GET(*sd, SdIor2);
      // diffuse_brdf "oren_nayar": initOrenNayar's A / B as the object holds
      // them (shinydiffuse.cc:170-176)
      s.oren_nayar = GET(*sd, SdOrenNayar) ? 1 : 0;
      s.oren_nayar_a = GET(*sd, SdOrenNayarA);
      s.oren_nayar_b = GET(*sd, SdOrenNayarB);
    } else if (s.bsdf_flags == BSDF_EMIT) {
      // lightMat_t is defined in a .cc (simple.cc:36-70): read lightCol and
      // doubleSided back through its virtual emit()
      s.type = YK_MAT_LIGHT;
      renderState_t st;
      st.includeLights = true;
      surfacePoint_t sp;
      sp.N = vector3d_t(0, 0, 1);
      const color_t front = m->emit(st, sp, vector3d_t(0, 0, 1));
      const color_t back = m->emit(st, sp, vector3d_t(0, 0, -1));
      put3(s.color, front.R, front.G, front.B);
      s.double_sided = !back.isBlack();
    } else {
      return unsupported("material type not on the GPU path");
    }
    if (yk_scene_add_material_state(ys, &s, &id) != YK_OK) return fail();
    ids[m] = id;
    return true;
  }
  bool fail() {
    Y_ERROR << integratorName << ": " << yk_last_error() << yendl;
    return false;
  }
  bool unsupported(const char* what) {
    Y_ERROR << integratorName << ": " << what << yendl;
    return false;
  }
  void release() {
    for (yk_device* d : devs) yk_device_close(d);
    if (ys) yk_scene_destroy(ys);
    devs.clear();
    ys = nullptr;
  }

  yk_render_params params;
  bool gpu_tree = false;  // "gpu_kdtree": device-built tree (yk_device_build_tree), documented tie-break
  int max_gpus = 0;       // "gpus": 0 = every GPU of the node
  yk_scene* ys = nullptr;
  std::vector<yk_device*> devs;  // one per GPU, the scene replicated on each
};

extern "C" {
YAFRAYPLUGIN_EXPORT void registerPlugin(renderEnvironment_t& render) {
  // same names as the CPU plugins: loaded after them, these win
  // (registerFactory is a map assignment, environment.cc:738-742)
  render.registerFactory("pathtracing", gpuTiledIntegrator_t::factory_path);
  render.registerFactory("directlighting", gpuTiledIntegrator_t::factory_direct);
  render.registerFactory("photonmapping", gpuTiledIntegrator_t::factory_photon);
}
}

__END_YAFRAY
