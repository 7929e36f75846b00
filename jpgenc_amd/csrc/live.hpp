// Live contexts and device groups, closed by the library at process exit.
//
// A context owns lane threads, HIP streams, device and pinned host memory; a group
// also owns RCCL communicators.  Left open at exit (a C caller that skips
// jpge_close, the facade's default context, a Python process whose objects outlive
// its own hooks), their teardown would otherwise run inside or after the static
// destructors of the HIP runtime, of RCCL and of a profiler's tool library, in an
// order nobody controls (round 3: a lane stream destroyed after rocprofv3's tool had
// finalised faulted the process).  The library therefore registers an exit handler
// (std::atexit) the first time a context opens, and again once RCCL is loaded:
// handlers run in reverse order of registration, so this one runs before the
// teardown of every runtime that was initialised before it, and closes what is still
// open: groups first (with their member contexts), then contexts.  It releases what
// they own (threads, streams, memory, communicators) but not the handles themselves,
// which the caller may still hold: a later jpge_close / jpge_group_close on them is a
// no-op, and any other call on them returns JPGE_E_ARG (a call still running on
// another thread is waited for first).  A forked child forgets the parent's objects
// (their threads do not exist in it).
#pragma once

struct jpge_ctx;
struct jpge_group;

namespace jpge {
void live_add(jpge_ctx* c);
void live_remove(jpge_ctx* c);
void live_add(jpge_group* g);
void live_remove(jpge_group* g);
// the exit handler's release of one handle (capi.cpp, group.cpp)
void live_release(jpge_ctx* c);
void live_release(jpge_group* g);
bool live_is_released(const void* handle);
void live_mark_released(const void* handle);
// register the exit handler again, after loading a runtime with its own teardown (RCCL)
void live_handler_after_load();
}  // namespace jpge
