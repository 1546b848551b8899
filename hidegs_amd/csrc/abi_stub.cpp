// abi_stub.cpp -- definitions of every entry point declared in include/hidegs.h.
//
// The rasterizer, binning and distCUDA2 kernels are not built (DESIGN.md,
// "Denials in force"), so every compute entry point validates nothing and
// returns HIDEGS_E_UNSUPPORTED with a message; callers (diff_gaussian_rasterization._C)
// turn that into a RuntimeError.  The library exists so the boundary -- symbol
// set, calling convention, error channel -- is real and tested end to end.
#include "../../include/hidegs.h"

#include <string>

namespace {
thread_local std::string g_last_error;
thread_local float g_hvar = 0.3f;
constexpr const char* kBlocked =
    "not implemented: the gfx950 rasterizer/knn kernels are not built pending a scope decision (DESIGN.md)";

int unsupported(const char* fn)
{
    g_last_error = std::string(fn) + ": " + kBlocked;
    return HIDEGS_E_UNSUPPORTED;
}
}  // namespace

extern "C" {

int hidegs_rasterize_forward(hidegs_alloc_fn, hidegs_alloc_fn, hidegs_alloc_fn, void*, int, int, int, const float*,
                             int, int, const int*, const int*, const float*, const int*, const float*, const float*,
                             const float*, const float*, const float*, const float*, float, const float*,
                             const float*, const float*, const float*, const float*, float, float, int, float*,
                             float*, int*, float*, float*, int, int*, int, void*, int* num_rendered)
{
    if (num_rendered) *num_rendered = 0;
    return unsupported("hidegs_rasterize_forward");
}

size_t hidegs_geometry_bytes(int) { return 0; }
size_t hidegs_binning_bytes(int) { return 0; }
size_t hidegs_image_bytes(int, int) { return 0; }

int hidegs_rasterize_backward(hidegs_alloc_fn, void*, int, int, int, int, const float*, const float*, int, int,
                              const int*, const int*, const float*, const int*, const float*, const float*,
                              const float*, const float*, const float*, const float*, const float*, float,
                              const float*, const float*, const float*, const float*, float, float, const int*, char*,
                              char*, char*, const float*, const float*, const float*, const float*, float*, float*,
                              float*, float*, float*, float*, float*, float*, float*, int, int, void*)
{
    return unsupported("hidegs_rasterize_backward");
}

int hidegs_mark_visible(int, const float*, const float*, const float*, unsigned char*, void*)
{
    return unsupported("hidegs_mark_visible");
}

int hidegs_dist_cuda2(hidegs_alloc_fn, void*, int, const float*, float*, void*)
{
    return unsupported("hidegs_dist_cuda2");
}
size_t hidegs_knn_scratch_bytes(int) { return 0; }

void hidegs_set_backward_hvar(float h_var) { g_hvar = h_var; }
float hidegs_get_backward_hvar(void) { return g_hvar; }

void hidegs_enable_stage_timing(int) {}
void hidegs_reset_stage_times(void) {}
int hidegs_stage_times(double* ms, long long* launches)
{
    for (int i = 0; i < HIDEGS_NUM_STAGES; i++) {
        if (ms) ms[i] = 0.0;
        if (launches) launches[i] = 0;
    }
    return 0;
}
const char* hidegs_stage_name(int stage) { return (stage >= 0 && stage < HIDEGS_NUM_STAGES) ? "unused" : nullptr; }

const char* hidegs_last_error(void) { return g_last_error.c_str(); }
const char* hidegs_version(void) { return "hidegs-abi 0.2 (compute entry points unsupported)"; }

}  // extern "C"
