// Reference-backed ingest checker (test infrastructure, never shipped): the reference's own OBJ
// types and loader support code (include/OBJ_Loader.h + src/OBJ_Loader.cpp, compiled from where
// they lie under /root/reference by oracle/Makefile.ref) driving a verbatim-order restatement of
// OBJFileManager::LoadObjFile (src/OBJ_FileManager.cpp:10-70). OBJ_FileManager.cpp itself cannot be
// compiled here: its header includes DirectXMath.h, which the image lacks (no stand-ins are made).
// The function below follows it statement for statement — std::getline, the line minus its first
// character through a std::stringstream, `ss >> x >> y >> z` into objl::Vector3 positions, face
// indices decremented as unsigned ints — so the float parsing is the C++ library's, as in the
// reference.
//
//   ref_obj_ingest <file.obj> <out.bin>
// writes: u32 vertex count, u32 index count, vertex positions (3 x f32 each), indices (u32 each).
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "OBJ_Loader.h"

// OBJ_FileManager.cpp:10-70
static bool load_obj_file(const std::string& path, std::vector<objl::Vertex>& vertices,
                          std::vector<unsigned int>& indices) {
  std::ifstream file(path);
  if (!file.good()) return false;
  std::string str;
  unsigned int max_index = 0;
  while (std::getline(file, str)) {
    if (str.length() < 2) continue;
    std::string data = std::string(str.c_str() + 1);
    std::stringstream ss = std::stringstream(data);
    if (str[0] == 'v' && str[1] == ' ') {
      float x = 0.0f, y = 0.0f, z = 0.0f;  // the reference leaves them uninitialised (read only on
      ss >> x >> y >> z;                  // a failed extraction: not reached by the models)
      objl::Vertex v;
      v.Position = objl::Vector3(x, y, z);
      vertices.push_back(v);
    } else if (str[0] == 'f' && str[1] == ' ') {
      unsigned int i0 = 0, i1 = 0, i2 = 0;  // (as above)
      ss >> i0 >> i1 >> i2;
      i0--;
      i1--;
      i2--;
      unsigned int current_max = 0;
      if (i0 > i1 && i0 > i2) current_max = i0;
      if (i1 > i0 && i1 > i2) current_max = i1;
      if (i2 > i1 && i2 > i0) current_max = i2;
      if (current_max > max_index) max_index = current_max;
      indices.push_back(i0);
      indices.push_back(i1);
      indices.push_back(i2);
    } else {
      continue;
    }
  }
  return true;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s <file.obj> <out.bin>\n", argv[0]);
    return 2;
  }
  std::vector<objl::Vertex> v;
  std::vector<unsigned int> idx;
  if (!load_obj_file(argv[1], v, idx)) return 1;
  FILE* f = std::fopen(argv[2], "wb");
  if (!f) return 1;
  const unsigned int nv = (unsigned int)v.size(), ni = (unsigned int)idx.size();
  std::fwrite(&nv, 4, 1, f);
  std::fwrite(&ni, 4, 1, f);
  for (const objl::Vertex& x : v) {
    const float p[3] = {x.Position.X, x.Position.Y, x.Position.Z};
    std::fwrite(p, 4, 3, f);
  }
  if (ni) std::fwrite(idx.data(), 4, ni, f);
  std::fclose(f);
  return 0;
}
