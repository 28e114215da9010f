// fcg_sweep_totlag.hip -- the TotLag instantiations of the row-block sweep (fcg_sweep.hip) in a
// translation unit of their own, so that they can be compiled without the SLP vectorizer (see
// launch_sweep_h8_totlag in fcg_sweep.hip and the 4c_amd/Makefile rule).
#define FCG_SWEEP_TOTLAG_TU
#include "fcg_sweep.hip"
