// hipmock/hip/hip_fp16.h — TEST INFRASTRUCTURE ONLY: rccl/rccl.h includes this header; the host build of the group
// merge (tests/cpp/hipmock/hip/hip_runtime.h) uses no half types.
#pragma once
