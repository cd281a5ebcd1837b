// probe-only: render an XML scene through libyafaraycore into a float RGBA buffer
#include <core_api/scene.h>
#include <core_api/environment.h>
#include <core_api/imagefilm.h>
#include <yafraycore/xmlparser.h>
#include <yafraycore/memoryIO.h>
#include <cstdio>
#include <vector>
using namespace yafaray;
int main(int argc, char** argv){
  renderEnvironment_t env; env.loadPlugins(argv[2]);
  yafout.setMasterVerbosity(VL_MUTE);
  scene_t* scene = new scene_t(); env.setScene(scene);
  paraMap_t render; if(!parse_xml_file(argv[1], scene, &env, render)) return 1;
  int w=320,h=240; render.getParam("width",w); render.getParam("height",h);
  std::vector<float> buf(size_t(w)*h*4);
  memoryIO_t out(w,h,buf.data());
  if(!env.setupScene(*scene, render, out)) return 2;
  scene->render();
  FILE* f=fopen(argv[3],"wb"); fwrite(buf.data(),4,buf.size(),f); fclose(f);
  return 0;
}
