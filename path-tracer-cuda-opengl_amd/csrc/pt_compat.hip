// pt_compat.hip — the compat-mode wide render kernels (renderKernelWF<S, false, true>) in a
// translation unit of their own, compiled without the main unit's -mllvm --enable-post-misched=0
// (see the launcher at the end of pt_device.hip's kernels and DESIGN.md section 6).
#define PT_TU_COMPAT 1
#include "pt_device.hip"
