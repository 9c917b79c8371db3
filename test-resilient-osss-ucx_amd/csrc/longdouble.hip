// longdouble.hip -- x87 80-bit extended reduce-to-all combine (placeholder).
#include "combine.hpp"

namespace osgpu {

hipError_t launch_longdouble(int, void *, const void *const *, int, size_t, hipStream_t)
{
    return hipErrorNotSupported;
}

}  // namespace osgpu
