package ai.foremast.metrics.k8s.starter;

import org.springframework.boot.actuate.autoconfigure.security.servlet.EndpointRequest;
import org.springframework.boot.autoconfigure.AutoConfiguration;
import org.springframework.boot.autoconfigure.condition.ConditionalOnClass;
import org.springframework.boot.autoconfigure.condition.ConditionalOnMissingBean;
import org.springframework.boot.autoconfigure.condition.ConditionalOnWebApplication;
import org.springframework.context.annotation.Bean;
import org.springframework.core.annotation.Order;
import org.springframework.security.config.annotation.web.builders.HttpSecurity;
import org.springframework.security.web.SecurityFilterChain;

/**
 * When Spring Security is on the classpath: the actuator endpoints Prometheus
 * and the kubectl plugins call ({@code prometheus}, {@code health},
 * {@code k8s-metrics}) plus {@code /metrics} are reachable without a login;
 * CSRF is dropped for them when {@code k8s.metrics.disable-csrf} is set.
 */
@AutoConfiguration
@ConditionalOnWebApplication(type = ConditionalOnWebApplication.Type.SERVLET)
@ConditionalOnClass(name = "org.springframework.security.web.SecurityFilterChain")
public class ActuatorAccessConfig {

    @Bean
    @Order(0)
    @ConditionalOnMissingBean(name = "foremastActuatorChain")
    public SecurityFilterChain foremastActuatorChain(HttpSecurity http, K8sMetricsProperties props) throws Exception {
        http.requestMatchers(m -> m.requestMatchers(
                        EndpointRequest.to("prometheus", "health", "k8s-metrics"),
                        new org.springframework.security.web.util.matcher.AntPathRequestMatcher("/metrics")))
                .authorizeRequests(a -> a.anyRequest().permitAll());
        if (props.isDisableCsrf()) {
            http.csrf().disable();
        }
        return http.build();
    }
}
