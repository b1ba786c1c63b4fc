! slate_amd Fortran 2003 module: ISO_C_BINDING interfaces to the C ABI of
! libslate_amd_c.so (include/slate_amd/c_api.h).
!
! Reference parity: the reference generates a Fortran module from its C API
! (tools/fortran/generate_fortran_module.py, used by examples/fortran/
! ex05_blas.f90).  Here the module is written by hand against the smaller
! slate_amd C ABI: every routine is the by-value C function, so Fortran
! callers pass scalars normally (VALUE) and arrays by reference.  Integers
! are 64-bit (c_int64_t); character flags are single c_char values; info is
! the function result (0 = success).
!
! Build:   flang -c slate_amd.f90                (produces slate_amd.mod)
! Link:    -L<repo>/slate_amd -lslate_amd_c -lpython3.x
module slate_amd
    use iso_c_binding
    implicit none

    interface
        integer(c_int) function slate_amd_initialize() bind(C, name="slate_amd_initialize")
            import :: c_int
        end function

        subroutine slate_amd_finalize() bind(C, name="slate_amd_finalize")
        end subroutine

        ! ---------------------------------------------------------------- BLAS-3
        integer(c_int) function slate_dgemm(transa, transb, m, n, k, alpha, a, lda, b, ldb, beta, c, ldc) &
                bind(C, name="slate_dgemm")
            import :: c_int, c_int64_t, c_double, c_char
            character(kind=c_char), value :: transa, transb
            integer(c_int64_t), value :: m, n, k, lda, ldb, ldc
            real(c_double), value :: alpha, beta
            real(c_double), intent(in) :: a(lda, *), b(ldb, *)
            real(c_double), intent(inout) :: c(ldc, *)
        end function

        integer(c_int) function slate_sgemm(transa, transb, m, n, k, alpha, a, lda, b, ldb, beta, c, ldc) &
                bind(C, name="slate_sgemm")
            import :: c_int, c_int64_t, c_float, c_char
            character(kind=c_char), value :: transa, transb
            integer(c_int64_t), value :: m, n, k, lda, ldb, ldc
            real(c_float), value :: alpha, beta
            real(c_float), intent(in) :: a(lda, *), b(ldb, *)
            real(c_float), intent(inout) :: c(ldc, *)
        end function

        integer(c_int) function slate_dtrsm(side, uplo, transa, diag, m, n, alpha, a, lda, b, ldb) &
                bind(C, name="slate_dtrsm")
            import :: c_int, c_int64_t, c_double, c_char
            character(kind=c_char), value :: side, uplo, transa, diag
            integer(c_int64_t), value :: m, n, lda, ldb
            real(c_double), value :: alpha
            real(c_double), intent(in) :: a(lda, *)
            real(c_double), intent(inout) :: b(ldb, *)
        end function

        ! -------------------------------------------------------------- Cholesky
        integer(c_int) function slate_dpotrf(uplo, n, a, lda) bind(C, name="slate_dpotrf")
            import :: c_int, c_int64_t, c_double, c_char
            character(kind=c_char), value :: uplo
            integer(c_int64_t), value :: n, lda
            real(c_double), intent(inout) :: a(lda, *)
        end function

        integer(c_int) function slate_dpotrs(uplo, n, nrhs, a, lda, b, ldb) bind(C, name="slate_dpotrs")
            import :: c_int, c_int64_t, c_double, c_char
            character(kind=c_char), value :: uplo
            integer(c_int64_t), value :: n, nrhs, lda, ldb
            real(c_double), intent(in) :: a(lda, *)
            real(c_double), intent(inout) :: b(ldb, *)
        end function

        integer(c_int) function slate_dposv(uplo, n, nrhs, a, lda, b, ldb) bind(C, name="slate_dposv")
            import :: c_int, c_int64_t, c_double, c_char
            character(kind=c_char), value :: uplo
            integer(c_int64_t), value :: n, nrhs, lda, ldb
            real(c_double), intent(inout) :: a(lda, *), b(ldb, *)
        end function

        integer(c_int) function slate_dpotri(uplo, n, a, lda) bind(C, name="slate_dpotri")
            import :: c_int, c_int64_t, c_double, c_char
            character(kind=c_char), value :: uplo
            integer(c_int64_t), value :: n, lda
            real(c_double), intent(inout) :: a(lda, *)
        end function

        ! -------------------------------------------------------------------- LU
        integer(c_int) function slate_dgetrf(m, n, a, lda, ipiv) bind(C, name="slate_dgetrf")
            import :: c_int, c_int64_t, c_double
            integer(c_int64_t), value :: m, n, lda
            real(c_double), intent(inout) :: a(lda, *)
            integer(c_int64_t), intent(out) :: ipiv(*)
        end function

        integer(c_int) function slate_dgetrs(trans, n, nrhs, a, lda, ipiv, b, ldb) bind(C, name="slate_dgetrs")
            import :: c_int, c_int64_t, c_double, c_char
            character(kind=c_char), value :: trans
            integer(c_int64_t), value :: n, nrhs, lda, ldb
            real(c_double), intent(in) :: a(lda, *)
            integer(c_int64_t), intent(in) :: ipiv(*)
            real(c_double), intent(inout) :: b(ldb, *)
        end function

        integer(c_int) function slate_dgesv(n, nrhs, a, lda, ipiv, b, ldb) bind(C, name="slate_dgesv")
            import :: c_int, c_int64_t, c_double
            integer(c_int64_t), value :: n, nrhs, lda, ldb
            real(c_double), intent(inout) :: a(lda, *), b(ldb, *)
            integer(c_int64_t), intent(out) :: ipiv(*)
        end function

        ! ------------------------------------------------------- least squares
        integer(c_int) function slate_dgels(trans, m, n, nrhs, a, lda, b, ldb) bind(C, name="slate_dgels")
            import :: c_int, c_int64_t, c_double, c_char
            character(kind=c_char), value :: trans
            integer(c_int64_t), value :: m, n, nrhs, lda, ldb
            real(c_double), intent(inout) :: a(lda, *), b(ldb, *)
        end function

        ! ------------------------------------------------------ eigen / SVD / norm
        integer(c_int) function slate_dsyev(jobz, uplo, n, a, lda, w) bind(C, name="slate_dsyev")
            import :: c_int, c_int64_t, c_double, c_char
            character(kind=c_char), value :: jobz, uplo
            integer(c_int64_t), value :: n, lda
            real(c_double), intent(inout) :: a(lda, *)
            real(c_double), intent(out) :: w(*)
        end function

        integer(c_int) function slate_dgesvd(jobu, jobvt, m, n, a, lda, s, u, ldu, vt, ldvt) &
                bind(C, name="slate_dgesvd")
            import :: c_int, c_int64_t, c_double, c_char
            character(kind=c_char), value :: jobu, jobvt
            integer(c_int64_t), value :: m, n, lda, ldu, ldvt
            real(c_double), intent(inout) :: a(lda, *)
            real(c_double), intent(out) :: s(*), u(ldu, *), vt(ldvt, *)
        end function

        real(c_double) function slate_dlange(norm, m, n, a, lda) bind(C, name="slate_dlange")
            import :: c_int64_t, c_double, c_char
            character(kind=c_char), value :: norm
            integer(c_int64_t), value :: m, n, lda
            real(c_double), intent(in) :: a(lda, *)
        end function
    end interface
end module slate_amd
