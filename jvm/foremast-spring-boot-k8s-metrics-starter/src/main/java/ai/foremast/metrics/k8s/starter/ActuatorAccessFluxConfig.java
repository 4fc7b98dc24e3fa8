package ai.foremast.metrics.k8s.starter;

import org.springframework.boot.autoconfigure.AutoConfiguration;
import org.springframework.boot.autoconfigure.condition.ConditionalOnClass;
import org.springframework.boot.autoconfigure.condition.ConditionalOnMissingBean;
import org.springframework.boot.autoconfigure.condition.ConditionalOnWebApplication;
import org.springframework.context.annotation.Bean;
import org.springframework.core.annotation.Order;
import org.springframework.security.config.web.server.ServerHttpSecurity;
import org.springframework.security.web.server.SecurityWebFilterChain;
import org.springframework.security.web.server.util.matcher.ServerWebExchangeMatchers;

/**
 * {@link ActuatorAccessConfig} for reactive applications: with Spring Security
 * on the classpath, the endpoints Prometheus and the kubectl plugins call
 * ({@code /actuator/prometheus}, {@code /actuator/health}, {@code /actuator/info},
 * {@code /actuator/k8s-metrics/**}, {@code /metrics}) are reachable without a
 * login; CSRF is dropped for them when {@code k8s.metrics.disable-csrf} is set.
 * Every other path keeps the application's own security chain.
 */
@AutoConfiguration
@ConditionalOnWebApplication(type = ConditionalOnWebApplication.Type.REACTIVE)
@ConditionalOnClass(name = "org.springframework.security.web.server.SecurityWebFilterChain")
public class ActuatorAccessFluxConfig {

    @Bean
    @Order(0)
    @ConditionalOnMissingBean(name = "foremastActuatorFluxChain")
    public SecurityWebFilterChain foremastActuatorFluxChain(ServerHttpSecurity http, K8sMetricsProperties props) {
        http.securityMatcher(ServerWebExchangeMatchers.pathMatchers("/actuator/prometheus", "/actuator/health",
                        "/actuator/info", "/actuator/k8s-metrics/**", "/metrics"))
                .authorizeExchange(a -> a.anyExchange().permitAll());
        if (props.isDisableCsrf()) {
            http.csrf(c -> c.disable());
        }
        return http.build();
    }
}
