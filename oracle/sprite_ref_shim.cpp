// ORACLE (test infrastructure only): an extern "C" entry to the reference's own
// SPRITE kernel get_rg2s_cpp (igm/cython_compiled/cpp_sprite_assignment.h:1-8),
// which is compiled from the reference source file itself by `make -C oracle ref`
// into oracle/_ref/libsprite_ref.so.  Nothing of the reference is copied here.
#include "cpp_sprite_assignment.h"

extern "C" void sprite_ref_get_rg2s(float* crds, int n_struct, int n_bead, int n_regions, int* copies_num,
                                    float* rg2s, int* copy_idxs, int* min_struct) {
    get_rg2s_cpp(crds, n_struct, n_bead, n_regions, copies_num, rg2s, copy_idxs, min_struct);
}
