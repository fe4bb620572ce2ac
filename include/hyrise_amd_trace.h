/*
 * Operator tracing entry points of the MI355X execution layer (a separate header from hyrise_amd.h so that the kernel
 * translation units do not depend on it).
 *
 * Replaces nothing in the reference; it fills the reference's documented extension point for per-operator
 * measurements, OperatorPerformanceData (src/lib/operators/operator_performance_data.hpp:10-15, stamped by
 * AbstractOperator::execute, abstract_operator.cpp:30-53): the host operators bracket their stream work with two
 * timing events and report the device time between them next to the walltime.
 */
#ifndef HYRISE_AMD_TRACE_H
#define HYRISE_AMD_TRACE_H

#include <stdint.h>

#include "hyrise_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hy_event_s* hy_event_t;

/* A timing event (hipEventCreate). */
hy_status hy_event_create(hy_event_t* event);
/* Records the event on the stream (NULL: the null stream). */
hy_status hy_event_record(hy_event_t event, hy_stream_t stream);
/* Nanoseconds between two recorded events; waits for `stop` to complete. */
hy_status hy_event_elapsed_ns(hy_event_t start, hy_event_t stop, uint64_t* ns);
hy_status hy_event_destroy(hy_event_t event);

#ifdef __cplusplus
}
#endif

#endif
