! Fortran example / test (reference: examples/fortran/ex05_blas.f90):
! dgemm, LU solve and Cholesky solve through the slate_amd module.
program ex_fortran
    use slate_amd
    implicit none
    integer(c_int64_t), parameter :: n = 40, nrhs = 3
    real(c_double) :: a(n, n), a0(n, n), s(n, n), b(n, nrhs), b0(n, nrhs), c(n, nrhs), r(n, nrhs)
    integer(c_int64_t) :: ipiv(n), i
    integer(c_int) :: info, info2, info3
    real(c_double) :: err, err2, err3

    call random_seed()
    call random_number(a0)
    call random_number(b0)
    do i = 1, n
        a0(i, i) = a0(i, i) + real(n, c_double)
    end do
    if (slate_amd_initialize() /= 0) stop 2

    ! C = A0 * B0
    c = 0
    info3 = slate_dgemm('N', 'N', n, nrhs, n, 1.0_c_double, a0, n, b0, n, 0.0_c_double, c, n)
    err3 = maxval(abs(c - matmul(a0, b0)))
    print '(a, i0, a, es10.3)', 'dgemm info=', info3, ' error=', err3

    ! LU solve
    a = a0
    b = b0
    info = slate_dgesv(n, nrhs, a, n, ipiv, b, n)
    r = matmul(a0, b) - b0
    err = maxval(abs(r))
    print '(a, i0, a, es10.3)', 'dgesv info=', info, ' residual=', err

    ! SPD solve with S = A0 A0^T + n I
    s = matmul(a0, transpose(a0))
    do i = 1, n
        s(i, i) = s(i, i) + real(n, c_double)
    end do
    a = s
    b = b0
    info2 = slate_dposv('L', n, nrhs, a, n, b, n)
    r = matmul(s, b) - b0
    err2 = maxval(abs(r))
    print '(a, i0, a, es10.3)', 'dposv info=', info2, ' residual=', err2

    call slate_amd_finalize()
    if (info /= 0 .or. info2 /= 0 .or. info3 /= 0 .or. err > 1e-9 .or. err2 > 1e-8 .or. err3 > 1e-10) stop 1
end program ex_fortran
