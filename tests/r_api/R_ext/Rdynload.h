/* see tests/r_api/R.h: declarations only, for the shim's compile check */
#ifndef BRR_TEST_RDYNLOAD_H
#define BRR_TEST_RDYNLOAD_H
#include <R.h>
#ifdef __cplusplus
extern "C" {
#endif
typedef void *(*DL_FUNC)(void);
typedef struct { const char *name; DL_FUNC fun; int numArgs; } R_CallMethodDef;
typedef struct _DllInfo DllInfo;
int R_registerRoutines(DllInfo *, const void *, const R_CallMethodDef *, const void *, const void *);
Rboolean R_useDynamicSymbols(DllInfo *, Rboolean);
#ifdef __cplusplus
}
#endif
#endif
