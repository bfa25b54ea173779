#include <Python.h>
int main(int argc, char **argv) {
    if (argc < 2) return 2;
    wchar_t *prog = Py_DecodeLocale(argv[0], NULL);
    Py_SetProgramName(prog);
    Py_Initialize();
    wchar_t **wargv = PyMem_RawMalloc(sizeof(wchar_t *) * (size_t)(argc - 1));
    for (int i = 1; i < argc; ++i) wargv[i - 1] = Py_DecodeLocale(argv[i], NULL);
    PySys_SetArgvEx(argc - 1, wargv, 0);
    FILE *f = fopen(argv[1], "r");
    if (!f) return 3;
    int rc = PyRun_SimpleFileEx(f, argv[1], 1);
    if (Py_FinalizeEx() < 0) rc = 120;
    return rc ? 1 : 0;
}
