// fp32 instantiation of the general-stencil row march (pds_sm_impl.hpp)
#include "pds_sm_impl.hpp"

namespace pcs {
template int sm_slots<float>();
template int sm_launch<float>(const pcs_pds2d_args* a, RowBands rb, hipStream_t st);
}  // namespace pcs
