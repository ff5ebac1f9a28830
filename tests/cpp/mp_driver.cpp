// Test driver for the MotionPlanning.hpp drop-in: the call sequence of the planner's Rock
// component (initPython -> runPyFunction -> sizePyArray -> returnPyArray* -> shutDownPython).
//   mp_driver <module> <function>   (prints what it read, one "key value..." per line)
#include <cstdio>

#include "../../include/MotionPlanning.hpp"

int main(int argc, char** argv)
{
    MotionPlanning_lib::MotionPlanning mp;
    PyObject* mod = mp.initPython(argv[1]);
    if (!mod) return 2;
    char dir[] = "/nonexistent/map";
    mp.runPyFunction(argv[2], mod, 10.0, 12.0, 30.5, 40.5, 0.25, dir, 0.1, 5.0);
    int n = 0, m = 0;
    char vpath[] = "finalRoverPath", vhead[] = "finalRoverHeading", vasg[] = "assignment", vbad[] = "notAnArray";
    mp.sizePyArray(n, vpath, mod);
    mp.sizePyArray(m, vasg, mod);
    double* path = nullptr;
    double* head = nullptr;
    int* asg = nullptr;
    int* bad = nullptr;
    mp.returnPyArrayDouble(2, vpath, path, mod);
    mp.returnPyArrayDouble(1, vhead, head, mod);
    mp.returnPyArrayInt(1, vasg, asg, mod);
    mp.returnPyArrayInt(1, vpath, bad, mod);  // wrong dtype -> nullptr
    PyObject* fm = PyObject_GetAttrString(mod, "FM_FILE");
    std::printf("FM_FILE %s\n", fm ? PyUnicode_AsUTF8(fm) : "?");
    Py_XDECREF(fm);
    std::printf("SIZES %d %d\n", n, m);
    std::printf("PATH");
    for (int i = 0; path && i < 3 * n; ++i) std::printf(" %.17g", path[i]);
    std::printf("\nHEAD");
    for (int i = 0; head && i < n; ++i) std::printf(" %.17g", head[i]);
    std::printf("\nASG");
    for (int i = 0; asg && i < m; ++i) std::printf(" %d", asg[i]);
    std::printf("\nBAD %s\n", bad ? "nonnull" : "null");
    return mp.shutDownPython(mod);
}
