// fp64 instantiation of the general-stencil row march (pds_sm_impl.hpp)
#include "pds_sm_impl.hpp"

namespace pcs {
template int sm_slots<double>();
template int sm_launch<double>(const pcs_pds2d_args* a, RowBands rb, hipStream_t st);
}  // namespace pcs
