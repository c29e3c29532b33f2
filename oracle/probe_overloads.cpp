// Which pow/sqrt/abs overloads the reference's hot-path calls bind to.
//
// The reference's translation unit is Main.cpp -> Renderer.hpp, whose line 4
// includes IOHelpers.hpp; IOHelpers.hpp:5-9 defines STB_IMAGE_WRITE_IMPLEMENTATION
// and STB_IMAGE_IMPLEMENTATION and includes stb_image_write.h / stb_image.h.  Their
// implementation sections include <stdlib.h> and <math.h> (public stb source; the
// reference's third_party/stb submodule is empty here).  Under libstdc++ those are
// wrapper headers that do `using std::abs; using std::pow; using std::sqrt;`, so by
// the time Renderer.hpp:6-8 includes SingleThreadPathTracer.hpp, TaskBasedPathTracer.hpp
// and SceneGenerators.hpp, the unqualified calls
//   pow(float, float)   SingleThreadPathTracer.hpp:58-59,75-76  TaskBasedPathTracer.hpp:137-138,155-156
//   sqrt(float)         SingleThreadPathTracer.hpp:66,68,82,84  TaskBasedPathTracer.hpp:146,148,162,164
//   abs(float)          SceneGenerators.hpp:34
// find the float overloads.  Build with -DSPT_PROBE_STB=0 to see the resolution a
// TU without the stb headers would get (double pow/sqrt, ::abs(int)).
//
// Test infrastructure (tests/test_oracle_kat.py::test_overload_probe); prints one line
// per call and exits 0.
#ifndef SPT_PROBE_STB
#define SPT_PROBE_STB 1
#endif
#if SPT_PROBE_STB
#include <stdlib.h>  // stb_image.h / stb_image_write.h implementation sections
#include <math.h>
#endif
#include <cmath>
#include <cstdio>
#include <type_traits>

// the reference's call shapes, at global scope like SampleColorRefractive
static float probe_c = 0.3f, probe_z = 1.25f;
#define KIND(e) (std::is_same<decltype(e), float>::value ? "float" : std::is_same<decltype(e), double>::value ? "double" : "int")

int main()
{
    std::printf("pow(float,float) -> %s\n", KIND(pow(1.f - probe_c, 5.f)));
    std::printf("sqrt(float) -> %s\n", KIND(sqrt(1.f - probe_c * probe_c)));
    std::printf("abs(float) -> %s\n", KIND(abs(probe_z)));
    std::printf("abs(1.25f)*0.85f = %a\n", (double)((abs(probe_z)) * 0.85f));
    return 0;
}
