// MotionPlanning.cpp -- implementation of the drop-in MotionPlanning_lib::MotionPlanning
// (include/MotionPlanning.hpp).  Written against the CPython embedding API and the buffer
// protocol; the planner it loads reaches the GPU solver through the FastMarching drop-in.
#include "../../include/MotionPlanning.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <string>

namespace
{
// the package directory holding FastMarching/: env MOTIONPLANNING_FM_PATH, else relative to this
// library (<pkg>/lib/libmotionplanning.so -> <pkg>)
std::string fm_package_dir()
{
    const char* env = std::getenv("MOTIONPLANNING_FM_PATH");
    if (env && *env) return env;
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(&fm_package_dir), &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        for (int up = 0; up < 2; ++up) {
            const size_t k = p.find_last_of('/');
            if (k == std::string::npos) return "";
            p.resize(k);
        }
        return p;
    }
    return "";
}

// arrays handed out by returnPyArray*: kept alive (and their buffers held) until shutdown
struct Held {
    PyObject* obj;
    Py_buffer view;
};
std::vector<Held> g_held;

// borrow a C-contiguous buffer of pModule.<name> with the given struct format and rank
bool get_array(PyObject* pModule, const char* name, const char* fmt, int nDim, Py_buffer* view, PyObject** obj)
{
    *obj = pModule ? PyObject_GetAttrString(pModule, name) : nullptr;
    if (!*obj) {
        if (PyErr_Occurred()) PyErr_Print();
        std::cerr << "'" << name << "' is not an attribute of the module" << std::endl;
        return false;
    }
    if (PyObject_GetBuffer(*obj, view, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) {
        PyErr_Print();
        std::cerr << "'" << name << "' is not a C-contiguous array" << std::endl;
        Py_DECREF(*obj);
        return false;
    }
    const char* f = view->format ? view->format : "B";
    if (*f == '@' || *f == '=' || *f == '<') ++f;  // native / little-endian prefixes
    const bool fmt_ok = fmt[0] == 'd' ? (std::strcmp(f, "d") == 0)
                                      : ((std::strcmp(f, "i") == 0 || std::strcmp(f, "l") == 0) && view->itemsize == 4);
    if (!fmt_ok || (nDim > 0 && view->ndim != nDim)) {
        std::cerr << "'" << name << "': expected a " << nDim << "-d " << (fmt[0] == 'd' ? "float64" : "int32")
                  << " array, got format '" << (view->format ? view->format : "?") << "' ndim " << view->ndim
                  << std::endl;
        PyBuffer_Release(view);
        Py_DECREF(*obj);
        return false;
    }
    return true;
}
}  // namespace

using namespace MotionPlanning_lib;

PyObject* MotionPlanning::initPython(char* pyName)
{
    std::cout << "Loading python file named '" << pyName << "'...";
    if (!Py_IsInitialized()) Py_Initialize();
    // the MI355X FastMarching package shadows any other one on the path
    const std::string pkg = fm_package_dir();
    if (!pkg.empty()) {
        PyObject* path = PySys_GetObject("path");  // borrowed
        PyObject* dir = PyUnicode_DecodeFSDefault(pkg.c_str());
        if (path && dir) PyList_Insert(path, 0, dir);
        Py_XDECREF(dir);
    }
    PyObject* name = PyUnicode_DecodeFSDefault(pyName);
    PyObject* module = name ? PyImport_Import(name) : nullptr;
    Py_XDECREF(name);
    if (module) {
        std::cout << " done" << std::endl;
    } else {
        PyErr_Print();
        std::cerr << "failed to load " << pyName << std::endl;
    }
    return module;
}

void MotionPlanning::runPyFunction(char pyFunctionName[], PyObject* pModule, double xm, double ym, double xr,
                                   double yr, double initHeading, char mapDirectory[], double resolution, double size)
{
    std::cout << "Running function '" << pyFunctionName << "'..." << std::endl;
    PyObject* func = pModule ? PyObject_GetAttrString(pModule, pyFunctionName) : nullptr;
    if (!func || !PyCallable_Check(func)) {
        if (PyErr_Occurred()) PyErr_Print();
        std::cout << "... ERROR when calling function " << pyFunctionName << std::endl;
        Py_XDECREF(func);
        return;
    }
    PyObject* ret = PyObject_CallFunction(func, "dddddsdd", xm, ym, xr, yr, initHeading, mapDirectory, resolution, size);
    if (!ret) {
        PyErr_Print();
        std::cout << "... ERROR when calling function " << pyFunctionName << std::endl;
    } else {
        std::cout << "... done" << std::endl;
    }
    Py_XDECREF(ret);
    Py_DECREF(func);
}

void MotionPlanning::sizePyArray(int& size, char pyVariableName[], PyObject* pModule)
{
    size = 0;
    PyObject* obj = pModule ? PyObject_GetAttrString(pModule, pyVariableName) : nullptr;
    if (!obj) {
        if (PyErr_Occurred()) PyErr_Print();
        return;
    }
    Py_buffer view;
    if (PyObject_GetBuffer(obj, &view, PyBUF_STRIDES | PyBUF_FORMAT) == 0) {
        if (view.ndim >= 1) size = (int)view.shape[0];
        PyBuffer_Release(&view);
    } else {
        PyErr_Print();
    }
    Py_DECREF(obj);
}

void MotionPlanning::returnPyArrayDouble(int nDim, char pyVariableName[], double*& dVariable, PyObject* pModule)
{
    std::cout << "Loading python variable named '" << pyVariableName << "'... ";
    dVariable = nullptr;
    Held h;
    if (!get_array(pModule, pyVariableName, "d", nDim, &h.view, &h.obj)) {
        std::cout << "failed" << std::endl;
        return;
    }
    dVariable = static_cast<double*>(h.view.buf);
    g_held.push_back(h);
    std::cout << "done" << std::endl;
}

void MotionPlanning::returnPyArrayInt(int nDim, char pyVariableName[], int*& iVariable, PyObject* pModule)
{
    std::cout << "Loading python variable named '" << pyVariableName << "'... ";
    iVariable = nullptr;
    Held h;
    if (!get_array(pModule, pyVariableName, "i", nDim, &h.view, &h.obj)) {
        std::cout << "failed" << std::endl;
        return;
    }
    iVariable = static_cast<int*>(h.view.buf);
    g_held.push_back(h);
    std::cout << "done" << std::endl;
}

int MotionPlanning::shutDownPython(PyObject* pModule)
{
    std::cout << "Finalizing python interpreter...";
    for (auto& h : g_held) {
        PyBuffer_Release(&h.view);
        Py_DECREF(h.obj);
    }
    g_held.clear();
    Py_XDECREF(pModule);
    Py_FinalizeEx();
    std::cout << " done" << std::endl;
    return 0;
}
