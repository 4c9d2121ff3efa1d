/* _npsel -- hands numpy's own argsort routine for float64 (the ArrFuncs entry np.argsort
 * dispatches to, kind="quicksort") to libmdroll as a plain C function pointer, so the
 * rollout's tie hand-shake can apply the reference's selection rule np.argsort(-q)
 * (U/MultiDismantler_torch.py:725,769) on the host thread without entering Python. */
#define PY_SSIZE_T_CLEAN
#define NPY_NO_DEPRECATED_API NPY_2_0_API_VERSION
#include <Python.h>
#include <numpy/arrayobject.h>

static PyObject* argsort_f64(PyObject* self, PyObject* args) {
  (void)self;
  (void)args;
  PyArray_Descr* d = PyArray_DescrFromType(NPY_DOUBLE);
  if (!d) return NULL;
  PyArray_ArgSortFunc* f = PyDataType_GetArrFuncs(d)->argsort[NPY_QUICKSORT];
  Py_DECREF(d);
  if (!f) {
    PyErr_SetString(PyExc_RuntimeError, "numpy has no float64 argsort");
    return NULL;
  }
  return PyLong_FromVoidPtr((void*)f);
}

static PyMethodDef methods[] = {
    {"argsort_f64", argsort_f64, METH_NOARGS, "address of numpy's float64 quicksort argsort (ArrFuncs)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_npsel", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__npsel(void) {
  import_array();
  return PyModule_Create(&mod);
}
