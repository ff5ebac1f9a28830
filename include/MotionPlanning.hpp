// MotionPlanning.hpp -- drop-in for the reference's C++ entry points
// (esa-prl/planning-motion_planning src/MotionPlanning.hpp:17-26, namespace MotionPlanning_lib).
//
// Same class, method names and signatures.  The reference embeds the Python planner
// (Coupled_motion_planner.py), whose cost-to-go solves import `FastMarching.FastMarching` /
// `FastMarching.FastMarching3D`; this implementation puts the MI355X drop-in FastMarching package
// (planning-motion_planning_amd/FastMarching, C ABI include/eikonal.h underneath) first on the
// embedded interpreter's sys.path, so the planner's solves run on the GPU unchanged.
//
// Differences from the reference, all on the safe side:
//  * the Rock `base/*` headers are included only when present (__has_include), numpy's C API
//    is not needed (arrays are read through the buffer protocol);
//  * returnPyArrayDouble / returnPyArrayInt check dtype ('d' / 32-bit int), C-contiguity and
//    rank, and return nullptr (with a message) instead of a pointer of the wrong type;
//  * object references are released (the reference leaks them); the arrays handed out stay
//    alive until shutDownPython, as in the reference.
#ifndef _MOTIONPLANNING_LIBRARIES_HPP_
#define _MOTIONPLANNING_LIBRARIES_HPP_

#if defined(__has_include)
#if __has_include(<base/samples/RigidBodyState.hpp>)
#include <base/samples/RigidBodyState.hpp>
#include <base/samples/DistanceImage.hpp>
#include <base/samples/Frame.hpp>
#include <base/Waypoint.hpp>
#endif
#endif

#include <Python.h>

#include <cmath>
#include <iostream>
#include <vector>

namespace MotionPlanning_lib
{
class MotionPlanning
{
   public:
    // Start the interpreter (if not running), put the FastMarching drop-in first on sys.path
    // (env MOTIONPLANNING_FM_PATH, else the build-time package directory) and import `pyName`.
    // NULL (and the Python error printed) on failure.  MotionPlanning.cpp:5-29.
    PyObject* initPython(char* pyName);
    // pModule.<pyFunctionName>(xm, ym, xr, yr, initHeading, mapDirectory, resolution, size);
    // errors are printed, as in the reference (:31-53).
    void runPyFunction(char pyFunctionName[], PyObject* pModule, double xm, double ym, double xr, double yr,
                       double initHeading, char mapDirectory[], double resolution, double size);
    // size = first dimension of the array pModule.<pyVariableName> (:55-64); 0 if it is not one.
    void sizePyArray(int& size, char pyVariableName[], PyObject* pModule);
    // Borrowed pointer into the float64 array pModule.<pyVariableName> (:65-76).
    void returnPyArrayDouble(int nDim, char pyVariableName[], double*& dVariable, PyObject* pModule);
    // Borrowed pointer into the int32 array pModule.<pyVariableName> (:79-90).
    void returnPyArrayInt(int nDim, char pyVariableName[], int*& iVariable, PyObject* pModule);
    // Release the module and the arrays handed out, finalize the interpreter; 0 (:93-100).
    int shutDownPython(PyObject* pModule);
};

}  // namespace MotionPlanning_lib

#endif
