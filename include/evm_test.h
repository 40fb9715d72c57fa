/* Test-only entry points of libevm: NOT part of the product ABI (include/evm.h).
 *
 * Fault injection for the atomicity tests (tests/test_gpu_server_atomic.py).
 * Every call returns EVM_EINVAL unless the process environment holds
 * EVM_TEST_HOOKS=1, so a product caller cannot switch a correctness check off.
 */
#ifndef EVM_TEST_H
#define EVM_TEST_H

#include "evm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* mode 0: no fault (the default);
 * mode 1: the sort-path phase of a split ingest fails (EVM_ENOMEM), so the
 *         ingest must roll back what its LDS phase staged;
 * mode 2: K5 leaves out its check against the stored rows, so a redelivered
 *         stored timestamp reaches the merge as a new row and the merge's
 *         guard must return EVM_ESTATE with nothing committed. */
int evm_test_fault(evm_ctx* ctx, int mode);

#ifdef __cplusplus
}
#endif

#endif
