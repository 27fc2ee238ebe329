/* C library interface to OINK (reference oink/library.h:22-27, library.cpp:26-98).
 *
 * The reference's header names these mrmpi_* while the implementation
 * defines oink_*; here header and library agree on oink_*. The communicator
 * argument is the opaque handle from MR_comm_world() (NULL = the same job
 * communicator, bootstrapped from torchrun-style RANK / WORLD_SIZE /
 * LOCAL_RANK / MASTER_ADDR / MASTER_PORT; one process per GPU, RCCL). */
#ifndef MRHIP_OINK_LIBRARY_H
#define MRHIP_OINK_LIBRARY_H

#ifdef __cplusplus
extern "C" {
#endif

void oink_open(int argc, char **argv, void *communicator, void **ptr);
void oink_open_no_mpi(int argc, char **argv, void **ptr);
void oink_close(void *ptr);
void oink_file(void *ptr, char *str);
/* run one command line; returns the command name (free with oink_free) or NULL */
char *oink_command(void *ptr, char *str);
void oink_free(void *ptr);

#ifdef __cplusplus
}
#endif
#endif
